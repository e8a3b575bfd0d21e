set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || exit $rc
for D in fp32 bf16; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2_$D -o run -- python3 bench.py --steps 10 --warmup 3 --dtype $D --gemm blas > gpurun_out/prof2_$D.log 2>&1 || exit 1
done
