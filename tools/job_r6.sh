set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
J=j53
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/${J}_tests.log 2>&1 || { tail -60 gpurun_out/${J}_tests.log; exit 1; }
tail -2 gpurun_out/${J}_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${J}_smoke.log 2>&1 || { tail -30 gpurun_out/${J}_smoke.log; exit 1; }
tail -1 gpurun_out/${J}_smoke.log
timeout -k 10 400 python3 -u bench.py > gpurun_out/${J}_bench.log 2>&1 || { tail -30 gpurun_out/${J}_bench.log; exit 1; }
tail -1 gpurun_out/${J}_bench.log | cut -c1-160
