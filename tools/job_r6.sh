set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_h3p_gpu.py tests/test_layer_prog_gpu.py > gpurun_out/j7_tests.log 2>&1 || { tail -40 gpurun_out/j7_tests.log; exit 1; }
tail -2 gpurun_out/j7_tests.log
timeout -k 10 400 python3 -u tools/bench_h3p.py --rounds 3 > gpurun_out/j7_gemm.log 2>&1 || { tail -20 gpurun_out/j7_gemm.log; exit 1; }
cut -c1-220 gpurun_out/j7_gemm.log
timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 5 --ab "rf_on,rf_off" --ab-rounds 8 > gpurun_out/j7_ab.log 2>&1 || { tail -20 gpurun_out/j7_ab.log; exit 1; }
tail -1 gpurun_out/j7_ab.log
