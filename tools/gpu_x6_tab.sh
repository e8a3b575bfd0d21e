cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "splitk or x6_error" --timeout 120 --timeout-method thread > gpurun_out/t_x6.log 2>&1; rc=$?
tail -2 gpurun_out/t_x6.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/t_x6.log; exit $rc; }
timeout -k 10 300 python tools/bench_gemm_x6.py --ksplit ${KS:-0,1,2,4} --md gpurun_out/gemm_x6.md > gpurun_out/gemm_x6.log 2>&1 || { tail -20 gpurun_out/gemm_x6.log; exit 1; }
cut -c1-330 gpurun_out/gemm_x6.log
