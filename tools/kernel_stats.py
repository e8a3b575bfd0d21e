#!/usr/bin/env python3
"""Per-kernel time table from a rocprofv3 kernel-trace database (rocpd sqlite, ROCm 7.x).

    python tools/kernel_stats.py gpurun_out/prof_x/run_results.db [--steps N] [--top 30] [--md]

Rows: kernel (arguments stripped), dispatches, total ms, ms per step (--steps: the number of
training steps the traced program ran, warm-up included), mean us, share of all kernel time.
Buckets at the end: hand-written hs:: kernels, of which GEMM (gemm*), library GEMM (Cijk_ / hipBLASLt),
everything else.
"""
import argparse
import collections
import re
import sqlite3


def short(name, n=90):
    name = re.sub(r"\(.*", "", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tot = collections.Counter()
    cnt = collections.Counter()
    for name, dur in c.execute("select name, duration from kernels"):
        k = short(name)
        tot[k] += dur
        cnt[k] += 1
    allns = sum(tot.values())
    print("| kernel | calls/step | ms/step | avg us | share |")
    print("|---|---|---|---|---|")
    for k, ns in tot.most_common(a.top):
        print("| `%s` | %.1f | %.3f | %.1f | %.1f%% |" % (k, cnt[k] / a.steps, ns / 1e6 / a.steps, ns / cnt[k] / 1e3,
                                                    100.0 * ns / allns))
    b = collections.Counter()
    for k, ns in tot.items():
        if "hs::" in k or k.startswith(("sort_keys", "hs_")):
            b["hs:: (hand-written)"] += ns
            if "gemm" in k:
                b["  of which hs GEMM"] += ns
        elif k.startswith("Cijk") or "hipblaslt" in k.lower() or "gemm" in k.lower():
            b["library GEMM"] += ns
        else:
            b["other (torch, copies)"] += ns
    print("\n| bucket | ms/step | share |\n|---|---|---|")
    print("| all kernels | %.3f | 100%% |" % (allns / 1e6 / a.steps))
    for k, ns in b.items():
        print("| %s | %.3f | %.1f%% |" % (k, ns / 1e6 / a.steps, 100.0 * ns / allns))


if __name__ == "__main__":
    main()
