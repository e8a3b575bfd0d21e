set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
J=j20
bash tools/gpu.sh configs || exit 1
for W in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --emulate-world $W > gpurun_out/${J}_emu$W.log 2>&1 || { tail -20 gpurun_out/${J}_emu$W.log; exit 1; }
  tail -1 gpurun_out/${J}_emu$W.log | cut -c1-160
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${J}_t1.log 2>&1 || { tail -20 gpurun_out/${J}_t1.log; exit 1; }
tail -1 gpurun_out/${J}_t1.log | cut -c1-160
