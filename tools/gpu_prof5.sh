# kernel-trace profile of the fp32 bench (GEMM choices measured first in an untraced run, then loaded)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
for D in ${DTYPES:-fp32 bf16}; do
rm -f gpurun_out/choices_$D.json
timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 --dtype $D --gemm-choices gpurun_out/choices_$D.json > gpurun_out/b5_$D.log 2>&1 || exit 1
tail -1 gpurun_out/b5_$D.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5_$D -o run -- python3 bench.py --steps 10 --warmup 2 --dtype $D --gemm-choices gpurun_out/choices_$D.json > gpurun_out/prof5_$D.log 2>&1 || exit 1
python3 tools/prof_summary.py gpurun_out/prof5_$D/run_kernel_stats.csv 12 "BERT-base seq128 bs32, 1x MI355X, $D (kernel time per step)" > gpurun_out/prof5_$D.md
head -8 gpurun_out/prof5_$D.md
done
