cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_x6.log 2>&1; rc=$?
tail -2 gpurun_out/t_x6.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/t_x6.log; exit $rc; }
for s in 2048,2048,4096,1,0 3072,768,4096,1,0; do for w in 4 8; do for ab in 0 1; do
timeout -k 10 120 python3 tools/bench_gemm_x6.py --only $s,x6 --reps 30 --ablate $ab --waves $w 2>/dev/null || exit 1
done; done; done
timeout -k 10 300 python tools/bench_gemm_x6.py --ksplit 0,1,2,4 --md gpurun_out/gemm_x6.md > gpurun_out/gemm_x6.log 2>&1 || { tail -20 gpurun_out/gemm_x6.log; exit 1; }
grep wgrad gpurun_out/gemm_x6.log | cut -c1-330; tail -1 gpurun_out/gemm_x6.log
