"""One BERT-base product on the h3p engine (and on the h3 engine), repeated, for counter profiles:

    rocprofv3 --pmc ... -- python3 tools/prof_h3p_one.py [--shape qkv|wgrad|dgrad] [--iters 50]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402
from hetseq_amd.ops import h3p  # noqa: E402

SH = {"qkv": (4096, 2304, 768, 0, 1, 1), "dgrad": (4096, 768, 3072, 0, 0, 2), "wgrad": (2304, 768, 4096, 1, 0, 4),
      "ffn1": (4096, 3072, 768, 0, 1, 1),
      "odgrad": (4096, 768, 768, 0, 0, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="qkv")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--old", action="store_true")
    ap.add_argument("--rowmajor", action="store_true", help="also run row-major planes")
    a = ap.parse_args()
    M, N, K, ta, tb, ks = SH[a.shape]
    dev = torch.device("cuda", 0)
    A = torch.randn((K, M) if ta else (M, K), device=dev)
    B = torch.randn((N, K) if tb else (K, N), device=dev) * 0.05
    out = torch.empty(M, N, device=dev)
    ha, hb = h3p.split(A), h3p.split(B)
    am = (G.amax_of(A), G.amax_of(B))
    hr = (h3p.split(A, blk=False), h3p.split(B, blk=False)) if a.rowmajor else None
    for _ in range(a.iters):
        h3p.gemm(ha, hb, ta, tb, out=out, ksplit=ks)
        if hr:
            h3p.gemm(hr[0], hr[1], ta, tb, out=out, ksplit=ks)
        if a.old:
            G._hip_gemm(A, B, ta, tb, out, fp32="h3", ksplit=ks, amax=am)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
