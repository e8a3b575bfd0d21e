# controlled A/B of environment variants on one box (each variant run twice, interleaved)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
for rep in 1 2; do for cfg in "$@"; do
env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', d['dtype'], d['ms_per_step'], 'ms/step')"
done; done
