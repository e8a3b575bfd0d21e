set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_h3p_gpu.py tests/test_layer_prog_gpu.py > gpurun_out/t_bq.log 2>&1 || { tail -30 gpurun_out/t_bq.log; exit 1; }
tail -2 gpurun_out/t_bq.log
timeout -k 10 400 python3 bench.py --steps 30 --warmup 5 --ab bq_old,bq_new --ab-rounds 8 > gpurun_out/ab_bq3.log 2>&1 || { tail -20 gpurun_out/ab_bq3.log; exit 1; }
tail -1 gpurun_out/ab_bq3.log
