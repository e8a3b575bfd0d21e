# host-side cProfile of the bench loop (where the per-step host time goes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python3 -m cProfile -o gpurun_out/bench_fp32.prof bench.py --steps 40 --warmup 5 --gemm blas > gpurun_out/hp_fp32.log 2>&1 || exit 1
tail -1 gpurun_out/hp_fp32.log | cut -c1-200
