set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_h3p_gpu.py tests/test_layer_prog_gpu.py -k "attention or attn or layer_program or planes or bitwise" > gpurun_out/j5_tests.log 2>&1 || { tail -40 gpurun_out/j5_tests.log; exit 1; }
tail -2 gpurun_out/j5_tests.log
timeout -k 10 300 python3 -u tools/bench_producers.py --reps 30 > gpurun_out/j5_prod.log 2>&1 || { tail -20 gpurun_out/j5_prod.log; exit 1; }
grep attn gpurun_out/j5_prod.log
timeout -k 10 500 python3 -u bench.py --steps 10 --warmup 5 --ab "attf_pair+lead4,attf_tile+lead4,attb_occ1+lead4,attf_pair+lead3" --ab-rounds 8 > gpurun_out/j5_ab.log 2>&1 || { tail -20 gpurun_out/j5_ab.log; exit 1; }
tail -1 gpurun_out/j5_ab.log
timeout -k 10 600 python3 -u tools/h3p_census.py --steps 20 --every 10 --out gpurun_out/r6_h3_census.md > gpurun_out/j5_census.log 2>&1 || { tail -20 gpurun_out/j5_census.log; exit 1; }
tail -3 gpurun_out/j5_census.log
