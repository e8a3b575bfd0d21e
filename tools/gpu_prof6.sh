# kernel-trace profiles of the current engine: phase 1 fp32 / bf16 and phase 2 (seq 512, bs 8) fp32
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
prof() { N=$1; shift
timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 "$@" > gpurun_out/b6_$N.log 2>&1 || { tail -20 gpurun_out/b6_$N.log; exit 1; }
tail -1 gpurun_out/b6_$N.log | cut -c1-220
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6_$N -o run -- python3 bench.py --steps 10 --warmup 2 "$@" > gpurun_out/prof6_$N.log 2>&1 || { tail -20 gpurun_out/prof6_$N.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof6_$N/run_kernel_stats.csv 12 "BERT-base $*, 1x MI355X (kernel time per step)" > gpurun_out/prof6_$N.md || exit 1
head -9 gpurun_out/prof6_$N.md | tail -6
}
prof ph1_fp32 --dtype fp32 && prof ph1_bf16 --dtype bf16 && prof ph2_fp32 --dtype fp32 --seq-len 512 --batch 8 --max-pred 80
