# split-bf16 fp32 GEMM: numerics tests, then speed/error table, then the bench with each fp32 engine
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/t_x6.log 2>&1; rc=$?
tail -15 gpurun_out/t_x6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_gemm_x6.py --ksplit 0,1,2,4 --md gpurun_out/gemm_x6.md > gpurun_out/gemm_x6.log 2>&1 || { tail -20 gpurun_out/gemm_x6.log; exit 1; }
cat gpurun_out/gemm_x6.log | cut -c1-400
for e in x6 native; do
HETSEQ_FP32_GEMM=$e timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$e.log 2>&1 || { tail -20 gpurun_out/b_$e.log; exit 1; }
tail -1 gpurun_out/b_$e.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', d['ms_per_step'], 'ms/step; host', d['host_ms_per_step'], d['gemm_choices'])"
done
