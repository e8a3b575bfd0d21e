#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel: MFMA utilisation, achieved MFMA FLOP rate,
LDS bank-conflict rate.

usage: pmc_summary.py <run_counter_collection.csv> <title> [top_n]
Counters expected: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_{F32,BF16}, GRBM_GUI_ACTIVE,
SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE.  MI355X: 256 CUs x 4 SIMDs; 1 MOP = 512 FLOP.
"""
import csv
import sys
from collections import defaultdict

# sustained MFMA rates measured by tools/micro/mfma_peak.hip (profiles/r1_mfma_peak.md), TF/s
PEAK_F32 = 155.0
PEAK_BF16 = 2170.0


def main():
    path, title = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    per = defaultdict(lambda: defaultdict(float))
    ns = defaultdict(float)
    calls = defaultdict(set)
    gui = defaultdict(float)  # per dispatch: GRBM_GUI_ACTIVE is reported per XCD -> take the max
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        d = r["Dispatch_Id"]
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            gui[(k, d)] = max(gui[(k, d)], float(r["Counter_Value"]))
        else:
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if d not in calls[k]:
            calls[k].add(d)
            ns[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for (k, d), v in gui.items():
        per[k]["GRBM_GUI_ACTIVE"] += v
    rows = []
    for k, c in per.items():
        f32, b16 = 512.0 * c["SQ_INSTS_VALU_MFMA_MOPS_F32"], 512.0 * c["SQ_INSTS_VALU_MFMA_MOPS_BF16"]
        tf = (f32 + b16) / (ns[k] * 1e-9) / 1e12 if ns[k] else 0.0
        peak = PEAK_BF16 if b16 > f32 else PEAK_F32
        util = 100.0 * tf / peak
        lds = c["SQ_LDS_IDX_ACTIVE"]
        conf = 100.0 * c["SQ_LDS_BANK_CONFLICT"] / lds if lds else 0.0
        rows.append((ns[k], k, len(calls[k]), util, tf, conf))
    rows.sort(reverse=True)
    print("# %s\n" % title)
    print("Source: `rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 "
          "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace` over `bench.py --steps 3` "
          "(`%s`).  TF/s = MFMA FLOPs (512 x MFMA MOPS) / kernel time (counter runs serialise kernels, so times "
          "are indicative); %% of peak against the sustained rates measured by tools/micro/mfma_peak.hip "
          "(155 TF/s fp32, 2170 TF/s bf16); LDS conflict = bank-conflict cycles / LDS-active cycles.\n" % path)
    print("Split-bf16 fp32 GEMMs (`gemm_x6s_kernel<..., 6, ...>`) issue six bf16 products per fp32 product: their "
          "effective fp32 rate is the bf16 MFMA rate / 6 (last column).\n")
    print("| kernel | dispatches | total ms | MFMA TF/s | % of sustained MFMA peak | LDS conflict % | effective fp32 TF/s |\n"
          "|---|---|---|---|---|---|---|")
    for t, k, n, u, tf, cf in rows[:top]:
        eff = "%.1f" % (tf / 6.0) if "gemm_x6s_kernel" in k and ", 6," in k else ""
        print("| `%s` | %d | %.3f | %.1f | %.1f | %.1f | %s |" % (k.replace("|", "/")[:90], n, t / 1e6, tf, u, cf, eff))


if __name__ == "__main__":
    main()
