cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=${D:-fp32}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3_$D -o run -- python3 bench.py --steps 10 --warmup 3 --dtype $D --gemm blas > gpurun_out/prof3_$D.log 2>&1
