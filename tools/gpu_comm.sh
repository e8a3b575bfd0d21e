# native RCCL engine on one GPU (1-rank communicator), then the whole GPU suite and the 1-GPU bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_comm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/comm_tests.log 2>&1 || { tail -40 gpurun_out/comm_tests.log; exit 1; }
grep -E "PASS|FAIL|ERROR" gpurun_out/comm_tests.log | cut -c1-150
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1 || { tail -20 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log | cut -c1-400
