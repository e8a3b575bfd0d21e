# LayerNorm backward with 16 waves per block: numerics, then A/B against alt/ (4 waves per block)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_bert_gpu.py -x -q --timeout 120 --timeout-method thread -k "ln or layernorm or emb or bert or fused" -m gpu > gpurun_out/ln_tests.log 2>&1 || { tail -40 gpurun_out/ln_tests.log; exit 1; }
tail -2 gpurun_out/ln_tests.log
bash tools/gpu_ab_so.sh
