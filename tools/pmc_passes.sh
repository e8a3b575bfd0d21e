#!/usr/bin/env bash
# Counter passes over one program (run under gpurun from the repository root):
#   tools/pmc_passes.sh <tag> <program args...>
# Each pass is its own rocprofv3 run (counters are not split over passes); results are summarised
# per kernel by tools/pmc_summary.py into gpurun_out/pmc_<tag>.md.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
R=$PWD
tag=$1; shift
prog=$1; shift
case "$prog" in /*) ;; *) prog="$R/$prog" ;; esac
mkdir -p gpurun_out
export TMPDIR=/tmp
passes=(
  "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA"
  "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
)
dbs=()
i=0
for cs in "${passes[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $cs --kernel-trace -d "$R/gpurun_out/pmc_${tag}_$i" -o run -- python3 "$prog" "$@" \
     > "$R/gpurun_out/pmc_${tag}_$i.log" 2>&1) || { tail -20 "$R/gpurun_out/pmc_${tag}_$i.log"; exit 1; }
  db=$(ls "$R"/gpurun_out/pmc_${tag}_$i/run_results.db 2>/dev/null || find "$R/gpurun_out/pmc_${tag}_$i" -name '*.db' | head -1)
  dbs+=("$db")
done
python3 tools/pmc_summary.py "${dbs[@]}" --top 30 > "gpurun_out/pmc_${tag}.md" && cat "gpurun_out/pmc_${tag}.md"
