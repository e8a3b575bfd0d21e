set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_bert_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or bert" > gpurun_out/t_lpt.log 2>&1 || { tail -30 gpurun_out/t_lpt.log; exit 1; }
tail -1 gpurun_out/t_lpt.log
timeout -k 10 200 python3 tools/bench_attention.py > gpurun_out/lpt_attn.txt 2>&1 || { tail -20 gpurun_out/lpt_attn.txt; exit 1; }
grep "B=" gpurun_out/lpt_attn.txt
for i in 1 2 3; do for f in 0 1; do
HETSEQ_ATTN_BWD_DKV_FIRST=$f timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 > gpurun_out/lpt1_$f$i.log 2>&1 || { tail -20 gpurun_out/lpt1_$f$i.log; exit 1; }
python3 -c "import json; print('ph1 dkv_first=$f', json.loads(open('gpurun_out/lpt1_$f$i.log').read().strip().splitlines()[-1])['ms_per_step'])"
done; done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 4 --seq-len 512 --batch 8 --max-pred 80 > gpurun_out/lpt2.log 2>&1 || { tail -20 gpurun_out/lpt2.log; exit 1; }
python3 -c "import json; print('ph2', json.loads(open('gpurun_out/lpt2.log').read().strip().splitlines()[-1])['ms_per_step'])"
