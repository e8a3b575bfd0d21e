set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/probes/bf16_head_probe.py > gpurun_out/j18_probe.log 2>&1 || { tail -30 gpurun_out/j18_probe.log; exit 1; }
cat gpurun_out/j18_probe.log | grep -v "^|"
