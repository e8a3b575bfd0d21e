# split-bf16 fp32 attention: numerics, then controlled A/B (phase 1 and phase 2) against the exact-fp32 kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" -m gpu > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
bash tools/gpu_ab_env.sh HETSEQ_ATTN_FP32=x6 HETSEQ_ATTN_FP32=native || exit 1
BENCH_ARGS="--seq-len 512 --batch 8 --max-pred 80" bash tools/gpu_ab_env.sh HETSEQ_ATTN_FP32=x6 HETSEQ_ATTN_FP32=native
