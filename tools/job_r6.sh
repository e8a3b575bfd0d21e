set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
J=j26
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_layer_prog_gpu.py tests/test_h3p_gpu.py -m gpu -k "attn or attention or layer or h3p" > gpurun_out/${J}_tests.log 2>&1 || { tail -60 gpurun_out/${J}_tests.log; exit 1; }
tail -2 gpurun_out/${J}_tests.log
timeout -k 10 300 python3 -u tools/bench_attn.py > gpurun_out/${J}_attn.log 2>&1 || { tail -20 gpurun_out/${J}_attn.log; exit 1; }
HS_AB_ROOT=$PWD/.abold timeout -k 10 300 python3 -u tools/bench_attn.py > gpurun_out/${J}_attn_old.log 2>&1 || { tail -20 gpurun_out/${J}_attn_old.log; exit 1; }
echo new; grep '^{' gpurun_out/${J}_attn.log; echo old; grep '^{' gpurun_out/${J}_attn_old.log
for R in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 > gpurun_out/${J}_bench_new$R.log 2>&1 || { tail -20 gpurun_out/${J}_bench_new$R.log; exit 1; }
  echo new; tail -1 gpurun_out/${J}_bench_new$R.log | cut -c1-140
  (cd .abold && timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5) > gpurun_out/${J}_bench_old$R.log 2>&1 || { tail -20 gpurun_out/${J}_bench_old$R.log; exit 1; }
  echo old; tail -1 gpurun_out/${J}_bench_old$R.log | cut -c1-140
done
