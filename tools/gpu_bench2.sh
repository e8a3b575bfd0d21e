# quick bench of both dtypes (committed GEMM tables, no new tuning)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
for D in ${DTYPES:-fp32 bf16}; do
timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --dtype $D ${BENCH_ARGS:-} > gpurun_out/b2_$D.log 2>&1 || exit 1
tail -1 gpurun_out/b2_$D.log | cut -c1-200
done
