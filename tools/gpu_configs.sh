# the other BASELINE.md configs that fit on one GPU: phase-2 seq512 bs8, update-freq 4, bf16
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
run() {  # name, args...
  n=$1; shift
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 "$@" > gpurun_out/cfg_$n.log 2>&1 || { echo "$n failed"; tail -20 gpurun_out/cfg_$n.log; return 1; }
  tail -1 gpurun_out/cfg_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['dtype'], d['ms_per_step'], 'ms/step', d['tokens_per_s'], 'tok/s host', d['host_ms_per_step'])"
}
run ph2_fp32 --seq-len 512 --batch 8 --max-pred 80 && run uf4_fp32 --update-freq 4 && run ph2_bf16 --seq-len 512 --batch 8 --max-pred 80 --dtype bf16 && run uf4_bf16 --update-freq 4 --dtype bf16
