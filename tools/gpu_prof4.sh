# kernel-trace profile of the bench for both dtypes with the committed GEMM tables
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
for D in fp32 bf16; do
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4_$D -o run -- python3 bench.py --steps 10 --warmup 3 --dtype $D --gemm blas > gpurun_out/prof4_$D.log 2>&1 || exit 1
done
timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --gemm blas > gpurun_out/b4_fp32.log 2>&1 || exit 1
tail -1 gpurun_out/b4_fp32.log | cut -c1-200
