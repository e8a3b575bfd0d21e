cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decoder or gemm" --timeout 120 --timeout-method thread > gpurun_out/t_dec.log 2>&1; rc=$?
tail -3 gpurun_out/t_dec.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/t_dec.log; exit $rc; }
bash tools/gpu_tests.sh || exit 1
rm -f gpurun_out/ch.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --gemm-choices gpurun_out/ch.json > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | cut -c1-200
grep -o 'decoder[^]]*' gpurun_out/ch.json | head; grep -A4 decoder gpurun_out/ch.json | head -30
