set -o pipefail
mkdir -p gpurun_out
HETSEQ_PLANES_SLICE_MAJOR=1 timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_bert_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or planes or bf16" > gpurun_out/t_sl.log 2>&1 || { tail -30 gpurun_out/t_sl.log; exit 1; }
tail -1 gpurun_out/t_sl.log
for i in 1 2 3; do for f in 0 1; do
HETSEQ_PLANES_SLICE_MAJOR=$f timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --dtype bf16 > gpurun_out/slb_$f$i.log 2>&1 || { tail -20 gpurun_out/slb_$f$i.log; exit 1; }
python3 -c "import json; print('bf16 planes slice_major=$f', json.loads(open('gpurun_out/slb_$f$i.log').read().strip().splitlines()[-1])['ms_per_step'])"
done; done
for i in 1 2; do
timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 > gpurun_out/slf_$i.log 2>&1 || { tail -20 gpurun_out/slf_$i.log; exit 1; }
python3 -c "import json; print('fp32 default', json.loads(open('gpurun_out/slf_$i.log').read().strip().splitlines()[-1])['ms_per_step'])"
done
