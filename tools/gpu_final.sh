# end-of-round evidence: PMC counters (fp32 / bf16), kernel profile of the fp32 step, smoke + 1-GPU bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
DTYPES="fp32 bf16" bash tools/gpu_pmc.sh || exit 1
DTYPES=fp32 bash tools/gpu_prof5.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
