#!/usr/bin/env python3
"""Per-step GPU busy vs wall time and the largest idle gaps from a rocprofv3 kernel trace.

usage: trace_gaps.py <run_kernel_trace.csv> [marker_kernel_substring]
One step = the kernels between the last two launches of the marker kernel (default: the fused Adam).
"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "adam_flat"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    step = rows[a + 1:b + 1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    print("step: wall %.3f ms, kernel busy %.3f ms, %d kernels" % ((t1 - t0) / 1e6, busy / 1e6, len(step)))
    gaps = []
    prev = rows[a]
    for r in step:
        g = int(r["Start_Timestamp"]) - int(prev["End_Timestamp"])
        if g > 2000:
            gaps.append((g / 1e3, prev["Kernel_Name"][:48], r["Kernel_Name"][:48]))
        prev = r
    print("idle gaps > 2us: total %.3f ms in %d gaps" % (sum(g for g, _, _ in gaps) / 1e3, len(gaps)))
    for g in sorted(gaps, reverse=True)[:15]:
        print("  %8.1f us  %s -> %s" % g)


if __name__ == "__main__":
    main()
