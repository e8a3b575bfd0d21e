cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
DP_CASES="--no-fused;--bucket-cap-mb 1000;--bucket-cap-mb 1;--no-fused --bucket-cap-mb 1" timeout -k 10 600 python tools/dp_bisect.py
