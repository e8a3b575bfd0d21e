# GEMM/kernel tests + bench (fused FFN epilogues)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/t_gemm.log 2>&1; rc=$?
tail -15 gpurun_out/t_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 > gpurun_out/b3_fp32.log 2>&1 || exit 1
tail -1 gpurun_out/b3_fp32.log | cut -c1-3000
