#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV into markdown (per-step ms).

usage: prof_summary.py <run_kernel_stats.csv> <steps> <title> > profiles/x.md
"""
import csv
import sys


def main():
    path, steps, title = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    gemm = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"].startswith("Cijk"))
    hsg = sum(float(r["TotalDurationNs"]) for r in rows if "hs::" in r["Name"] and "gemm" in r["Name"])
    hs = sum(float(r["TotalDurationNs"]) for r in rows if "hs::" in r["Name"])
    print("# %s\n" % title)
    print("Source: `rocprofv3 --kernel-trace --stats` (`%s`), %d profiled steps (incl. warmup).\n" % (path, steps))
    print("| bucket | ms/step | share |\n|---|---|---|")
    print("| all kernels | %.3f | 100%% |" % (tot / 1e6 / steps))
    print("| library GEMM (hipBLASLt Cijk_*) | %.3f | %.0f%% |" % (gemm / 1e6 / steps, 100 * gemm / tot))
    print("| hetseq_amd HIP kernels (hs::*) | %.3f | %.0f%% |" % (hs / 1e6 / steps, 100 * hs / tot))
    print("| of which hand-written GEMM (hs::gemm_*) | %.3f | %.0f%% |" % (hsg / 1e6 / steps, 100 * hsg / tot))
    print("| other (torch elementwise, copies) | %.3f | %.0f%% |\n" % ((tot - gemm - hs) / 1e6 / steps,
                                                                  100 * (tot - gemm - hs) / tot))
    print("| kernel | calls/step | avg us | ms/step |\n|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = r["Name"].replace("|", "/")[:110]
        print("| `%s` | %.1f | %.1f | %.3f |" % (name, int(r["Calls"]) / steps, float(r["AverageNs"]) / 1e3,
                                             float(r["TotalDurationNs"]) / 1e6 / steps))


if __name__ == "__main__":
    main()
