set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
J=j33
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/${J}_tests.log 2>&1 || { tail -60 gpurun_out/${J}_tests.log; exit 1; }
tail -2 gpurun_out/${J}_tests.log
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 5 --ab attds_on,attds_off --ab-rounds 8 > gpurun_out/${J}_ab.log 2>&1 || { tail -20 gpurun_out/${J}_ab.log; exit 1; }
tail -1 gpurun_out/${J}_ab.log
