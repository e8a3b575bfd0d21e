#!/usr/bin/env python3
"""h3 GEMM kernel variants on the BERT-base shapes, interleaved in one process (medians of rounds):
default (4 waves, two blocks per CU), 4 waves at three blocks per CU (168 VGPRs), against the
six-term x6 kernel.  usage: python tools/bench_h3_variants.py [--rounds R]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402
from tools.bench_gemm import SHAPES  # noqa: E402

VARIANTS = {"x6": ("x6", -1), "h3": ("h3", -1), "h3_occ3": ("h3", 1024)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    tot = {k: 0.0 for k in VARIANTS}
    for name, M, N, K, ta, tb in SHAPES:
        A = torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1
        B = torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1
        C = torch.empty(M, N, device="cuda")
        am = (G.amax_of(A), G.amax_of(B))
        ref = (A.t() if ta else A).double() @ (B.t() if tb else B).double()
        times = {k: [] for k in VARIANTS}
        errs = {}
        for r in range(a.rounds):
            for k, (eng, tile) in VARIANTS.items():
                f = lambda: G._hip_gemm(A, B, ta, tb, C, fp32=eng, tile=tile, amax=am)  # noqa: E731
                assert f()
                if r == 0:
                    torch.cuda.synchronize()
                    errs[k] = float((C.double() - ref).abs().max() / ref.abs().max())
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    f()
                e.record()
                e.synchronize()
                times[k].append(s.elapsed_time(e) * 1000 / a.iters)
        med = {k: sorted(v)[len(v) // 2] for k, v in times.items()}
        for k in tot:
            tot[k] += med[k]
        print("%-11s %5dx%5dx%5d " % (name, M, N, K) + "  ".join("%s %6.1fus (%.1e)" % (k, med[k], errs[k])
                                                                   for k in VARIANTS), flush=True)
    print("per-layer sum (us): " + "  ".join("%s %.1f" % kv for kv in tot.items()), flush=True)


if __name__ == "__main__":
    main()
