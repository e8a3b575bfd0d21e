# A/B eager vs --hip-graph on one box, interleaved (fp32 headline config)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention or layernorm or embedding" > gpurun_out/t_ab.log 2>&1 || { tail -20 gpurun_out/t_ab.log; exit 1; }
tail -1 gpurun_out/t_ab.log
for rep in 1 2; do
for g in "" "--hip-graph"; do
timeout -k 10 300 python bench.py --steps 60 --warmup 8 $g > gpurun_out/ab$rep$g.log 2>&1 || exit 1
tail -1 gpurun_out/ab$rep$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['dtype'], 'graph' if d['config']['hip_graph'] else 'eager', d['ms_per_step'])"
done
done
