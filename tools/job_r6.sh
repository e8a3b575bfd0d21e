set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
J=j17
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_kernels_gpu.py tests/test_bert_gpu.py -m gpu -k "planes or bf16 or decoder or mlm" > gpurun_out/${J}_tests.log 2>&1 || { tail -60 gpurun_out/${J}_tests.log; exit 1; }
tail -2 gpurun_out/${J}_tests.log
for R in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --dtype bf16 > gpurun_out/${J}_bench_new$R.log 2>&1 || { tail -20 gpurun_out/${J}_bench_new$R.log; exit 1; }
  echo new; tail -1 gpurun_out/${J}_bench_new$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_ms_per_step'], d['gemm_choices'])"
  (cd .abold && timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --dtype bf16) > gpurun_out/${J}_bench_old$R.log 2>&1 || { tail -20 gpurun_out/${J}_bench_old$R.log; exit 1; }
  echo old; tail -1 gpurun_out/${J}_bench_old$R.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_ms_per_step'])"
done
bash tools/gpu.sh prof bf16 r6e || exit 1
