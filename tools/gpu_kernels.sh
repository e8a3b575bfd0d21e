set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/t1_kernels.log 2>&1
rc=$?
tail -30 gpurun_out/t1_kernels.log
exit $rc
