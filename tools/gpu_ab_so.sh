# controlled A/B of two builds of the HIP module on one box: the tree's .so ("new") vs alt/ ("old")
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HETSEQ_GEMM_TUNE_MISSING=0
SO=hetseq_amd/_hip.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/new.so
for rep in 1 2; do for v in new old; do
if [ $v = new ]; then cp /tmp/new.so $SO; else cp alt/_hip.cpython-310-x86_64-linux-gnu.so $SO; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
tail -1 gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['dtype'], d['ms_per_step'], 'ms/step')"
done; done
