# full GPU test suite, then the bench for each dtype (committed GEMM tables)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit $rc
for d in ${DTYPES:-fp32 bf16}; do
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --dtype $d ${BENCH_ARGS:-} > gpurun_out/b_$d.log 2>&1 || exit 1
tail -1 gpurun_out/b_$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dtype'], d['ms_per_step'], 'ms/step; host', d['host_ms_per_step'])"
done
