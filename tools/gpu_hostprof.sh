# host-side cProfile of the timed bench loop (where the per-step host time goes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 600 python3 bench.py --steps 40 --warmup 5 --dtype ${D:-bf16} --host-profile gpurun_out/host_${D:-bf16}.prof > gpurun_out/hp.log 2>&1 || { tail -20 gpurun_out/hp.log; exit 1; }
tail -1 gpurun_out/hp.log | cut -c1-200
