# PMC counters per kernel (separate runs, kernel-trace only: never combined with sys/runtime traces)
# over the fp32 / bf16 bench steps with the committed GEMM choices (no measuring in the trace).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export HETSEQ_GEMM_TUNE_MISSING=0
for D in ${DTYPES:-fp32 bf16}; do
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$D -o run -- python3 $R/bench.py --steps 3 --warmup 2 --dtype $D > $R/gpurun_out/pmc_$D.log 2>&1 || { tail -30 $R/gpurun_out/pmc_$D.log; exit 1; }
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_$D/run_counter_collection.csv "BERT-base $D step: per-kernel MFMA / LDS counters (1x MI355X)" 25 > $R/gpurun_out/pmc_$D.md || exit 1
head -14 $R/gpurun_out/pmc_$D.md | tail -8
done
