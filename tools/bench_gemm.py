#!/usr/bin/env python3
"""GEMM microbenchmark: hand-written HIP MFMA kernel (each tile shape) vs the library, BERT-base shapes.

usage: python tools/bench_gemm.py [--dtype fp32]
Prints one line per (shape, engine): time (us) and TF/s.  Random operands (not zeros: DVFS).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402

SHAPES = [  # (name, M, N, K, ta, tb)
    ("qkv_fwd", 4096, 2304, 768, 0, 1), ("out_fwd", 4096, 768, 768, 0, 1), ("ffn1_fwd", 4096, 3072, 768, 0, 1),
    ("ffn2_fwd", 4096, 768, 3072, 0, 1), ("ffn2_dgrad", 4096, 3072, 768, 0, 0), ("ffn1_dgrad", 4096, 768, 3072, 0, 0),
    ("qkv_dgrad", 4096, 768, 2304, 0, 0), ("ffn1_wgrad", 3072, 768, 4096, 1, 0), ("ffn2_wgrad", 768, 3072, 4096, 1, 0),
    ("qkv_wgrad", 2304, 768, 4096, 1, 0), ("out_wgrad", 768, 768, 4096, 1, 0),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="0,1,2,4,5,6")
    ap.add_argument("--ablate", action="store_true", help="also time the no-global-load / no-staging builds")
    a = ap.parse_args()
    from hetseq_amd.runtime import gemm_tuning
    gemm_tuning.enable("fp32", tune_missing=False)
    torch.manual_seed(0)
    for name, M, N, K, ta, tb in SHAPES:
        A = torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1
        B = torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1
        C = torch.empty(M, N, device="cuda")
        fl = 2.0 * M * N * K
        At = A.t() if ta else A
        Bt = B.t() if tb else B
        t = timeit(lambda: torch.mm(At, Bt, out=C))
        line = ["%-11s %5dx%5dx%5d  blas %7.1fus %6.1fTF" % (name, M, N, K, t, fl / t / 1e6)]
        for tile in [int(x) for x in a.tiles.split(",")]:
            if not G._hip_gemm(A, B, ta, tb, C, tile=tile):
                continue
            t = timeit(lambda: G._hip_gemm(A, B, ta, tb, C, tile=tile))
            line.append("hip%d %7.1fus %6.1fTF" % (tile, t, fl / t / 1e6))
            for abl in (1, 2) if a.ablate else ():
                t = timeit(lambda: G._hip_gemm(A, B, ta, tb, C, tile=tile | (abl << 3)))
                line.append("a%d %6.1fTF" % (abl, fl / t / 1e6))
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
