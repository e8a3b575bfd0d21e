set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${1:-fp32}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$D -o run -- python3 bench.py --steps 10 --warmup 3 --dtype $D > gpurun_out/prof_$D.log 2>&1
rc=$?
tail -3 gpurun_out/prof_$D.log
find gpurun_out/prof_$D -name "*stats*" | head
exit $rc
