#!/usr/bin/env python3
"""fp32 GEMM engines on BERT-base shapes: speed and error against an fp64 oracle.

Engines: the library (hipBLASLt/rocBLAS via torch.mm, TunableOp table), the
hand-written exact-fp32 MFMA kernel, the split-bf16 kernel (x6: six bf16 products
per fp32 product, fp32-level error) and the per-tensor split-fp16 kernel (h3).
Error metric per engine: max over elements of |C - C64| / (|A| @ |B|), i.e. the
error in units of the magnitude sum the product accumulates (fp32 rounding of a
K-long dot product gives ~1e-7 on this scale).

usage: python tools/bench_gemm_x6.py [--md out.md]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402
from tools.bench_gemm import SHAPES, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--md", default=None)
    ap.add_argument("--ksplit", default="0", help="comma list of split-K settings for x6 (0 = automatic)")
    ap.add_argument("--only", default=None, help="profile mode: 'M,N,K,ta,tb,engine' run --reps times, nothing else")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--tr", type=int, default=-1, help="with --only: 1 transposed-read layout, 0 register transpose")
    ap.add_argument("--ks", type=int, default=1, help="with --only: split-K slices")
    ap.add_argument("--occ3", type=int, default=0, help="with --only: h3 kernel at three blocks per CU")
    a = ap.parse_args()
    if a.only:
        M, N, K, ta, tb, eng = a.only.split(",")
        M, N, K, ta, tb = int(M), int(N), int(K), int(ta), int(tb)
        A = torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1
        B = torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1
        C = torch.empty(M, N, device="cuda")
        am = (G.amax_of(A), G.amax_of(B)) if eng == "h3" else None
        f = (lambda: torch.mm(A.t() if ta else A, B.t() if tb else B, out=C)) if eng == "blas" else \
            (lambda: G._hip_gemm(A, B, ta, tb, C, fp32=eng, ksplit=a.ks,
                                 tile=(256 if a.tr == 1 else 512 if a.tr == 0 else 0) | (1024 if a.occ3 else 0),
                                 amax=am))
        t = timeit(f, a.reps)
        f()
        At, Bt = (A.t() if ta else A).double(), (B.t() if tb else B).double()
        err = float(((C.double() - At @ Bt).abs() / (At.abs() @ Bt.abs())).max())
        print("%s tr%d ks%d %dx%dx%d %.1fus %.1fTF err %.2e" % (eng, a.tr, a.ks, M, N, K, t,
                                                              2.0 * M * N * K / t / 1e6, err))
        return
    from hetseq_amd.runtime import gemm_tuning
    gemm_tuning.enable("fp32", tune_missing=False)
    torch.manual_seed(0)
    rows = []
    tot = {}
    for name, M, N, K, ta, tb in SHAPES:
        A = torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1
        B = torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1
        At = A.t() if ta else A
        Bt = B.t() if tb else B
        ref = At.double() @ Bt.double()
        mag = At.double().abs() @ Bt.double().abs()
        C = torch.empty(M, N, device="cuda")
        fl = 2.0 * M * N * K

        def err():
            return float(((C.double() - ref).abs() / mag).max())

        res = []
        t = timeit(lambda: torch.mm(At, Bt, out=C))
        res.append(("blas", t, err()))
        G._hip_gemm(A, B, ta, tb, C, fp32="native")
        t = timeit(lambda: G._hip_gemm(A, B, ta, tb, C, fp32="native"))
        res.append(("native", t, err()))
        for ks in [int(x) for x in a.ksplit.split(",")]:
            if not G._hip_gemm(A, B, ta, tb, C, fp32="x6", ksplit=ks):
                continue
            e = err()
            t = timeit(lambda: G._hip_gemm(A, B, ta, tb, C, fp32="x6", ksplit=ks))
            res.append(("x6" + ("" if ks == 0 else "/k%d" % ks), t, e))
        am = (G.amax_of(A), G.amax_of(B))  # producer-side |max| in the step: not timed here
        for ks in [int(x) for x in a.ksplit.split(",")]:
            if not G._hip_gemm(A, B, ta, tb, C, fp32="h3", ksplit=ks, amax=am):
                continue
            e = err()
            t = timeit(lambda: G._hip_gemm(A, B, ta, tb, C, fp32="h3", ksplit=ks, amax=am))
            res.append(("h3" + ("" if ks == 0 else "/k%d" % ks), t, e))
        line = "%-11s %5dx%5dx%5d " % (name, M, N, K) + "  ".join(
            "%s %6.1fus %6.1fTF err %.2e" % (n, t, fl / t / 1e6, e) for n, t, e in res)
        print(line, flush=True)
        rows.append((name, M, N, K, res))
        for n, t, e in res:
            tot[n] = tot.get(n, 0.0) + t
    print("per-layer sum (us): " + "  ".join("%s %.1f" % kv for kv in tot.items()), flush=True)
    if a.md:
        with open(a.md, "w") as f:
            f.write("# fp32 GEMM engines, BERT-base shapes, 1x MI355X\n\n")
            f.write("Source: `tools/bench_gemm_x6.py` (uniform [-1,1) operands, 20 timed reps).  err = max |C - C_fp64| "
                    "/ (|A|@|B|) elementwise.\n\n")
            names = [n for n, _, _ in rows[0][4]]
            f.write("| shape | M x N x K | " + " | ".join("%s us (TF/s) / err" % n for n in names) + " |\n")
            f.write("|---|---|" + "---|" * len(names) + "\n")
            for name, M, N, K, res in rows:
                d = {n: (t, e) for n, t, e in res}
                cells = []
                for n in names:
                    if n in d:
                        t, e = d[n]
                        cells.append("%.1f (%.0f) / %.1e" % (t, 2.0 * M * N * K / t / 1e6, e))
                    else:
                        cells.append("-")
                f.write("| %s | %dx%dx%d | %s |\n" % (name, M, N, K, " | ".join(cells)))
            f.write("\nSum over one layer's 11 GEMM shapes (us): " + ", ".join("%s %.1f" % kv for kv in tot.items()) + "\n")


if __name__ == "__main__":
    main()
