# smoke + the BASELINE configurations on one GPU (phase 1 / phase 2, fp32 / bf16, update-freq 4)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run() { timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
  tail -1 gpurun_out/cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['dtype'], 'seq', c['seq_len'], 'bs', c['per_gpu_batch'], 'uf', c['update_freq'], d['ms_per_step'], 'ms/step', d['seq_per_s'], 'seq/s')"; }
run --dtype fp32
run --dtype fp32 --update-freq 4
run --dtype fp32 --seq-len 512 --batch 8 --max-pred 80
run --dtype bf16 --seq-len 512 --batch 8 --max-pred 80
run --dtype bf16 --hip-graph
