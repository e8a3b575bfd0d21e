# A/B: weight-gradient side stream on/off (and side-stream split-K) on the fp32 / bf16 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
for D in ${DTYPES:-fp32}; do
for cfg in ${CFGS:-"HETSEQ_WGRAD_STREAM=0" "HETSEQ_SIDE_KSPLIT=auto" "HETSEQ_SIDE_KSPLIT=1" "HETSEQ_SIDE_KSPLIT=2" "HETSEQ_SIDE_KSPLIT=4"}; do
env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dtype $D > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$D', '$cfg', d['ms_per_step'], 'ms/step; host', d['host_ms_per_step'])"
done; done
