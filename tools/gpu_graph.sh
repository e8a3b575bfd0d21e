# HIP-graph tests + bench eager vs graph for both dtypes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python -m pytest tests/test_graph_gpu.py -x -q > gpurun_out/t_graph.log 2>&1; rc=$?
tail -30 gpurun_out/t_graph.log
[ $rc -eq 0 ] || exit $rc
for d in fp32 bf16; do
for g in "" "--hip-graph"; do
timeout -k 10 300 python bench.py --steps 50 --warmup 8 --dtype $d $g > gpurun_out/bg_$d$g.log 2>&1 || exit 1
tail -1 gpurun_out/bg_$d$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dtype'], d['config']['hip_graph'], d['ms_per_step'], 'ms/step; host', d['host_ms_per_step'])"
done
done
