set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_bert_gpu.py -x -q -m gpu > gpurun_out/t2_bert.log 2>&1; rc=$?
tail -15 gpurun_out/t2_bert.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/b_fused_fp32.log 2>&1 && tail -2 gpurun_out/b_fused_fp32.log &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-fused > gpurun_out/b_torch_fp32.log 2>&1 && tail -2 gpurun_out/b_torch_fp32.log &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --dtype bf16 > gpurun_out/b_fused_bf16.log 2>&1 && tail -2 gpurun_out/b_fused_bf16.log
