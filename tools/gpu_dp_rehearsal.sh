# rehearse the driver's multi-rank bench launch (torchrun, 2 ranks) on a 1-GPU box: gloo on GPU 0
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 3 --dist-backend gloo > gpurun_out/dp2.log 2>&1 || { tail -40 gpurun_out/dp2.log; exit 1; }
grep '"metric"' gpurun_out/dp2.log | cut -c1-400
