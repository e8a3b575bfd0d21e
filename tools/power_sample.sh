#!/usr/bin/env bash
# Power and engine clock of the GPU while bench.py runs (read-only rocm-smi queries from a second
# process).  Run under gpurun from the repository root:
#   bash tools/power_sample.sh [steps] [extra bench.py args...]   -> gpurun_out/power_*.log
# Prints one "t=<s> sclk=<MHz> power=<W>" line per 3-s sample, then the bench result line.
# profiles/r5_power.md was taken this way.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
steps=${1:-4000}; shift || true
timeout -k 10 300 python3 -u bench.py --steps "$steps" --warmup 5 "$@" > gpurun_out/power_bench.log 2>&1 &
BP=$!
i=0
while kill -0 "$BP" 2> /dev/null && [ $i -lt 60 ]; do
  sleep 3; i=$((i + 1))
  timeout -k 5 20 rocm-smi --showpower --showclocks > "gpurun_out/power_$i.log" 2>&1 || true
  echo "t=$((3 * i)) sclk=$(grep -i 'sclk clock level' "gpurun_out/power_$i.log" | head -1 | sed 's/.*(\(.*\)Mhz).*/\1/') power=$(grep -i 'Package Power' "gpurun_out/power_$i.log" | head -1 | sed 's/.*(W): *//')"
done
wait "$BP"; rc=$?
tail -1 gpurun_out/power_bench.log | cut -c1-200
exit $rc
