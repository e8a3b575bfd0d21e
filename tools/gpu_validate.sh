# round re-entry check: GPU test tier, smoke and the 1-GPU bench on the freshly built tree
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_v.log 2>&1 || { tail -20 gpurun_out/bench_v.log; exit 1; }
tail -1 gpurun_out/bench_v.log | cut -c1-400
timeout -k 10 300 python bench.py --dtype bf16 --hip-graph > gpurun_out/bench_v16.log 2>&1 || { tail -20 gpurun_out/bench_v16.log; exit 1; }
tail -1 gpurun_out/bench_v16.log | cut -c1-400
