# side-stream host cost A/B and HIP-graph replay, after the GPU test tier
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
bash tools/gpu_tests.sh || exit 1
for D in bf16 fp32; do for cfg in "HETSEQ_WGRAD_STREAM=1" "HETSEQ_WGRAD_STREAM=0"; do
env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dtype $D > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$D', '$cfg', d['ms_per_step'], 'ms/step; host', d['host_ms_per_step'])"
env $cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 --dtype $D --hip-graph > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$D graph', '$cfg', d['ms_per_step'], 'ms/step; host', d['host_ms_per_step'])"
done; done
