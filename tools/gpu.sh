#!/usr/bin/env bash
# One entry point for the GPU-box jobs (run under gpurun from the repository root):
#   tools/gpu.sh prof  [dtypes] [tag]  rocprofv3 kernel-trace stats of bench.py -> gpurun_out/prof_<tag>_<dtype>.md
#   tools/gpu.sh pmc   [dtypes] [tag]  MFMA / LDS counters per kernel          -> gpurun_out/pmc_<tag>_<dtype>.md
#   tools/gpu.sh bench [dtypes]        bench.py per dtype                      -> gpurun_out/bench_<dtype>.json
#   tools/gpu.sh tests [pytest args]   the GPU test suite (one process)        -> gpurun_out/gputests.log
#   tools/gpu.sh configs               every single-GPU BASELINE.md configuration -> gpurun_out/configs.jsonl
# Every GPU step runs under its own time limit; the first failure ends the job (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cmd=${1:-bench}; shift || true
case "$cmd" in
  prof)
    tag=${2:-cur}
    for D in ${1:-fp32 bf16}; do
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${tag}_$D" -o run \
        -- python3 "$R/bench.py" --steps 10 --warmup 4 --dtype "$D" > "$R/gpurun_out/prof_${tag}_$D.log" 2>&1) || { tail -20 "$R/gpurun_out/prof_${tag}_$D.log"; exit 1; }
      python3 tools/prof_summary.py "gpurun_out/prof_${tag}_$D/run_kernel_stats.csv" 14 "BERT-base $D ($tag)" > "gpurun_out/prof_${tag}_$D.md" || exit 1
      head -12 "gpurun_out/prof_${tag}_$D.md" | tail -6
    done ;;
  pmc)
    tag=${2:-cur}
    for D in ${1:-fp32 bf16}; do
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_${tag}_$D" -o run -- python3 "$R/bench.py" --steps 3 --warmup 2 --dtype "$D" > "$R/gpurun_out/pmc_${tag}_$D.log" 2>&1) || { tail -20 "$R/gpurun_out/pmc_${tag}_$D.log"; exit 1; }
      { echo "# BERT-base $D step: per-kernel MFMA / LDS counters ($tag; counters serialise the kernels)"; echo;
        python3 tools/pmc_summary.py "gpurun_out/pmc_${tag}_$D/run_counter_collection.csv" --top 25; } > "gpurun_out/pmc_${tag}_$D.md" || exit 1
      head -14 "gpurun_out/pmc_${tag}_$D.md" | tail -8
    done ;;
  bench)
    for D in ${1:-fp32 bf16}; do
      timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --dtype "$D" ${BENCH_ARGS:-} > "gpurun_out/bench_$D.log" 2>&1 || { tail -20 "gpurun_out/bench_$D.log"; exit 1; }
      tail -1 "gpurun_out/bench_$D.log" > "gpurun_out/bench_$D.json"; cut -c1-220 "gpurun_out/bench_$D.json"
    done ;;
  configs)  # the BASELINE.md table: every single-GPU configuration, one bench.py run each
    : > gpurun_out/configs.jsonl
    while read -r name args; do
      [ -z "$name" ] && continue
      timeout -k 10 400 python3 bench.py $args > "gpurun_out/cfg_$name.log" 2>&1 || { tail -20 "gpurun_out/cfg_$name.log"; exit 1; }
      echo "{\"config\": \"$name\", \"result\": $(tail -1 "gpurun_out/cfg_$name.log")}" >> gpurun_out/configs.jsonl
      echo "$name $(tail -1 "gpurun_out/cfg_$name.log" | cut -c1-160)"
    done <<'CFG'
ph1_fp32 --steps 30 --warmup 5
ph1_bf16 --steps 30 --warmup 5 --dtype bf16
ph1_bf16_graph --steps 30 --warmup 5 --dtype bf16 --hip-graph
ph1_fp32_uf4 --steps 10 --warmup 3 --update-freq 4
ph2_fp32 --steps 20 --warmup 4 --seq-len 512 --batch 8 --max-pred 80
ph2_bf16 --steps 20 --warmup 4 --seq-len 512 --batch 8 --max-pred 80 --dtype bf16
CFG
    ;;
  tests)
    timeout -k 10 1100 python3 -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread "$@" > gpurun_out/gputests.log 2>&1
    rc=$?; grep -E "passed|failed" gpurun_out/gputests.log | tail -3; exit $rc ;;
  *) echo "unknown job $cmd"; exit 2 ;;
esac
