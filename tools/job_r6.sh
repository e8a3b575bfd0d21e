set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/j3_tests.log 2>&1 || { tail -60 gpurun_out/j3_tests.log; exit 1; }
tail -3 gpurun_out/j3_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/j3_smoke.log 2>&1 || { tail -20 gpurun_out/j3_smoke.log; exit 1; }
tail -1 gpurun_out/j3_smoke.log
bash tools/gpu.sh prof fp32 r6b || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/j3_bench.log 2>&1 || { tail -20 gpurun_out/j3_bench.log; exit 1; }
tail -1 gpurun_out/j3_bench.log | cut -c1-300
