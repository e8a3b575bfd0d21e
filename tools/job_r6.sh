set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_h3p_gpu.py tests/test_layer_prog_gpu.py tests/test_bert_gpu.py tests/test_kernels_gpu.py -m gpu -k "gelu or h3p or layer or bert or planes" > gpurun_out/j13_tests.log 2>&1 || { tail -60 gpurun_out/j13_tests.log; exit 1; }
tail -2 gpurun_out/j13_tests.log
timeout -k 10 300 python3 -u tools/bench_h3p_epi.py --rounds 3 > gpurun_out/j13_epi.log 2>&1 && HS_AB_ROOT=$PWD/.abold timeout -k 10 300 python3 -u tools/bench_h3p_epi.py --rounds 3 > gpurun_out/j13_epi_old.log 2>&1 || { tail -20 gpurun_out/j13_epi.log; exit 1; }
grep '^{' gpurun_out/j13_epi.log; echo old; grep '^{' gpurun_out/j13_epi_old.log
for R in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > gpurun_out/j13_bench_new$R.log 2>&1 || { tail -20 gpurun_out/j13_bench_new$R.log; exit 1; }
  echo new; tail -1 gpurun_out/j13_bench_new$R.log | cut -c1-200
  (cd .abold && timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5) > gpurun_out/j13_bench_old$R.log 2>&1 || { tail -20 gpurun_out/j13_bench_old$R.log; exit 1; }
  echo old; tail -1 gpurun_out/j13_bench_old$R.log | cut -c1-200
done
