set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/bench_h3p_epi.py --rounds 4 > gpurun_out/j10_epi.log 2>&1 || { tail -20 gpurun_out/j10_epi.log; exit 1; }
grep '^{' gpurun_out/j10_epi.log
