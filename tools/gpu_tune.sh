# Refresh configs/tunableop/gfx950_$D.csv: tune every GEMM shape the bench hits, then re-bench with the table.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${D:-fp32}
mkdir -p gpurun_out/tune
export HETSEQ_TUNABLEOP_OUT=gpurun_out/tune/tunableop_$D.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=200
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --dtype $D --gemm blas > gpurun_out/tune_$D.log 2>&1 || exit 1
tail -1 gpurun_out/tune_$D.log | cut -c1-120
unset HETSEQ_TUNABLEOP_OUT
cp gpurun_out/tune/tunableop_${D}0.csv configs/tunableop/gfx950_$D.csv || exit 1
export HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --dtype $D --gemm blas > gpurun_out/tuned_$D.log 2>&1 || exit 1
tail -1 gpurun_out/tuned_$D.log | cut -c1-160
ls -la gpurun_out/tune
