# the round-end GPU test tier, as the driver runs it (one process, per-test timeout)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/t_gpu.log | awk '{print $NF, $1}' | sort | uniq -c | sort -rn | head -3
tail -3 gpurun_out/t_gpu.log
exit $rc
