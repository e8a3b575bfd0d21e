#!/usr/bin/env python3
"""BERT-base fp32 GEMM shapes: in-kernel-split x6s engine vs the ring plane kernel (1 GPU).

    python tools/bench_gemm_ring.py [--reps 50] [--shapes fwd,dgrad,wgrad]

Median of ``--reps`` back-to-back launches (after warm-up) per product, interleaved rounds.  The
ring kernel reads pre-split planes (the split is not timed: in the step the producers emit them).
Prints one markdown table: us per product and effective fp32 TF/s (2 M N K / t).
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402

SHAPES = [  # name, ta, tb, M, N, K
    ("qkv fwd", 0, 1, 4096, 2304, 768), ("out fwd", 0, 1, 4096, 768, 768), ("ffn1 fwd", 0, 1, 4096, 3072, 768),
    ("ffn2 fwd", 0, 1, 4096, 768, 3072), ("ffn2 dgrad", 0, 0, 4096, 3072, 768), ("ffn1 dgrad", 0, 0, 4096, 768, 3072),
    ("out dgrad", 0, 0, 4096, 768, 768), ("qkv dgrad", 0, 0, 4096, 768, 2304), ("qkv wgrad", 1, 0, 2304, 768, 4096),
    ("out wgrad", 1, 0, 768, 768, 4096), ("ffn1 wgrad", 1, 0, 3072, 768, 4096), ("ffn2 wgrad", 1, 0, 768, 3072, 4096),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1000.0)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--only", default=None, help="comma-separated product names (e.g. 'out fwd,qkv dgrad')")
    ap.add_argument("--engines", default="x6s,ring")
    ap.add_argument("--ks-sweep", action="store_true", help="also time the ring with K splits 1/2/4/8 (wgrads)")
    a = ap.parse_args()
    rows = []
    only = set(x.strip() for x in a.only.split(",")) if a.only else None
    eng = a.engines.split(",")
    for name, ta, tb, M, N, K in SHAPES:
        if only and name not in only:
            continue
        A = torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1
        B = torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1
        pa, pb = G.split(A), G.split(B)
        out = torch.empty(M, N, device="cuda")
        ks = G.ring_ksplit(M, N, K, bool(ta)) if ta else 1
        x6 = lambda: G._hip_gemm(A, B, ta, tb, out, ksplit=0)  # noqa: E731
        ring = lambda: G.gemm_planes(pa, pb, bool(ta), bool(tb), out, ksplit=ks, variant=G.RING)  # noqa: E731
        assert x6() and ring()
        tx, tr = [], []
        for _ in range(a.rounds):
            tx.append(timeit(x6, a.reps) if "x6s" in eng else float("nan"))
            tr.append(timeit(ring, a.reps) if "ring" in eng else float("nan"))
        t6, tg = min(tx), min(tr)
        fl = 2.0 * M * N * K
        rows.append((name, M, N, K, ks, t6, tg, fl / t6 / 1e6, fl / tg / 1e6))
        if a.ks_sweep and ta:
            sweep = {}
            for s_ in (1, 2, 4, 8):
                f_ = lambda: G.gemm_planes(pa, pb, bool(ta), bool(tb), out, ksplit=s_, variant=G.RING)  # noqa: E731
                if f_():
                    sweep[s_] = round(timeit(f_, a.reps), 1)
            print("ks sweep %s: %s" % (name, sweep), flush=True)
    print("| product | M | N | K | ring ks | x6s us | ring us | x6s fp32 TF/s | ring fp32 TF/s | ring bf16-MFMA TF/s |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print("| %s | %d | %d | %d | %d | %.1f | %.1f | %.0f | %.0f | %.0f |" % (r + (6 * r[8],)))
    t6 = sum(r[5] for r in rows)
    tg = sum(r[6] for r in rows)
    print("\nsum over one layer's 12 products: x6s %.1f us, ring %.1f us (%.2fx)" % (t6, tg, t6 / tg))


if __name__ == "__main__":
    main()
