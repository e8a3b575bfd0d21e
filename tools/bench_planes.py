#!/usr/bin/env python3
"""A/B of the GEMM engines on the BERT-base step's shapes (one process, interleaved rounds).

fp32 products: the in-kernel-split engine (gemm.hip ``x6s``) vs the bf16-plane engine
(gemm_planes.hip, P = 3) in each variant (0 = two LDS stages BK 32, 1 = one stage, 2 = two
stages BK 16), plus the library SGEMM.  bf16 products: the plane engine (P = 1) variants vs the
library.  Weight gradients at their split-K choices.  Prints a markdown table (median us).

    python tools/bench_planes.py [--rounds 7] [--out gpurun_out/bench_planes.md]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402
from hetseq_amd.ops._C import hip  # noqa: E402

T, H, I = 4096, 768, 3072
# (name, M, N, K, ta, tb): C[M,N] = op(A) op(B), the BERT-base per-layer products
SHAPES = [
    ("qkv fwd", T, 3 * H, H, False, True), ("out fwd", T, H, H, False, True), ("ffn1 fwd", T, I, H, False, True),
    ("ffn2 fwd", T, H, I, False, True),
    ("qkv dgrad", T, H, 3 * H, False, False), ("out dgrad", T, H, H, False, False),
    ("ffn1 dgrad", T, H, I, False, False), ("ffn2 dgrad", T, I, H, False, False),
    ("qkv wgrad", 3 * H, H, T, True, False), ("out wgrad", H, H, T, True, False),
    ("ffn1 wgrad", I, H, T, True, False), ("ffn2 wgrad", H, I, T, True, False),
]


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--out", default="gpurun_out/bench_planes.md")
    args = ap.parse_args()
    torch.manual_seed(0)
    rows = []
    for name, M, N, K, ta, tb in SHAPES:
        a = torch.randn((K, M) if ta else (M, K), device="cuda")
        b = torch.randn((N, K) if tb else (K, N), device="cuda")
        pa, pb = G.split(a), G.split(b)
        ab, bb = G.Planes.of_bf16(a.bfloat16()), G.Planes.of_bf16(b.bfloat16())
        out = torch.empty(M, N, device="cuda")
        outb = torch.empty(M, N, device="cuda", dtype=torch.float32 if ta else torch.bfloat16)
        ks = G._planes_ksplit(M, N, K, 3) if ta else 1
        ksb = G._planes_ksplit(M, N, K, 1) if ta else 1
        At, Bt = (a.t() if ta else a), (b.t() if tb else b)
        Atb, Btb = At.bfloat16(), Bt.bfloat16()
        fl = 2.0 * M * N * K
        cands = {
            "x6s": lambda: G._hip_gemm(a, b, ta, tb, out, fp32="x6", ksplit=4 if ta else 0),
            "sgemm": lambda: torch.mm(At, Bt, out=out),
            "bf16 lib": lambda: torch.mm(Atb, Btb),
        }
        for v in (0, 1, 2, 3, 4):
            cands["pl3 v%d" % v] = (lambda v=v: (hip().set_planes_variant(v), G.gemm_planes(pa, pb, ta, tb, out,
                                                                                          ksplit=ks)))
            cands["pl1 v%d" % v] = (lambda v=v: (hip().set_planes_variant(v), G.gemm_planes(ab, bb, ta, tb, outb,
                                                                                          ksplit=ksb)))
        times = {k: [] for k in cands}
        for _ in range(args.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn))
        hip().set_planes_variant(0)
        med = {k: statistics.median(v) for k, v in times.items()}
        rows.append((name, M, N, K, ks, med, fl))
        print(name, {k: round(v, 1) for k, v in med.items()}, flush=True)
    keys = list(rows[0][5].keys())
    lines = ["# GEMM engines on the BERT-base shapes (median us over %d interleaved rounds, 1x MI355X)" % args.rounds,
             "", "x6s = in-kernel split-bf16 (gemm.hip); pl3 = pre-split planes (gemm_planes.hip, P=3) variant "
             "0/1/2; pl1 = bf16 planes (P=1); sgemm / bf16 lib = torch.mm.  Effective fp32 TF/s of the best fp32 "
             "engine in the last column.", "",
             "| product | M | N | K | ks | " + " | ".join(keys) + " | best fp32 TF/s |",
             "|---|---|---|---|---|" + "---|" * len(keys) + "---|"]
    for name, M, N, K, ks, med, fl in rows:
        best = min(med[k] for k in med if k.startswith("pl3") or k in ("x6s", "sgemm"))
        lines.append("| %s | %d | %d | %d | %d | " % (name, M, N, K, ks) + " | ".join("%.1f" % med[k] for k in keys)
                     + " | %.0f |" % (fl / best / 1e6))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
