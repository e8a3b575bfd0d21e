set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
J=j27
for AB in "w2_ks4,w2_ks2,w2_ks8" "wo_ks2,wo_ks1,wo_ks4" "sideks_2,sideks_1,sideks_4" "lnw1,lnw0" "attf_auto,attf_pair"; do
  timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 5 --ab $AB --ab-rounds 6 > gpurun_out/${J}_ab.log 2>&1 || { tail -20 gpurun_out/${J}_ab.log; exit 1; }
  tail -1 gpurun_out/${J}_ab.log
done
