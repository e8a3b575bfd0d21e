cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=$((20000 + RANDOM % 10000))
timeout -k 10 300 python tools/dp_debug.py 0 $P > gpurun_out/dbg0.log 2>&1 &
timeout -k 10 300 python tools/dp_debug.py 1 $P > gpurun_out/dbg1.log 2>&1
wait
cat gpurun_out/dbg0.log | grep -v Warning | tail -30
