#!/usr/bin/env python3
"""LayerNorm backward and embedding-sort kernel times on the BERT-base shape (rows 4096, H 768).

    python tools/bench_ln.py [--reps 50]

Prints median us per call and the effective HBM rate of ln_bwd (dy, z read; dz, da written).
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import bert_ops  # noqa: E402


def timeit(fn, reps):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1000.0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    rows, H = 4096, 768
    dy = torch.randn(rows, H, device="cuda")
    z = torch.randn(rows, H, device="cuda")
    mean = torch.randn(rows, device="cuda")
    rstd = torch.rand(rows, device="cuda") + 0.5
    g = torch.randn(H, device="cuda")
    acc = (torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda"), torch.zeros(H, device="cuda"))
    t = timeit(lambda: bert_ops.ln_bwd(dy, z, mean, rstd, g, 0.1, 1, 1, 2, True, True, acc=acc), a.reps)
    print("ln_bwd (BDR, dz + da, accumulate): %.1f us = %.2f TB/s" % (t, 4 * rows * H * 4 / t / 1e6))
    t = timeit(lambda: bert_ops.ln_bwd(dy, z, mean, rstd, g, 0.0, 1, 1, 2, True, True, acc=acc), a.reps)
    print("ln_bwd (BDR, p = 0): %.1f us" % t)
    ids = torch.randint(0, 30522, (rows,), device="cuda")
    t = timeit(lambda: bert_ops.sort_keys(ids, 30522), a.reps)
    tt = timeit(lambda: torch.sort(ids, stable=True), a.reps)
    print("sort_keys 4096 keys: %.1f us (torch.sort %.1f us)" % (t, tt))


if __name__ == "__main__":
    main()
