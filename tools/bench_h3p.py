"""Isolated timing of the BERT-base fp32 products: the in-kernel-split h3 engine (gemm.hip, NT=4,
per-tensor scales) against the h3p engine (gemm_h3p.hip, pre-split block-scaled planes; blocked
plane layout, and row-major planes for comparison).

    python tools/bench_h3p.py [--json out.jsonl]

Interleaved rounds in one process (rule: A/B in one process); fp16-MFMA TF/s = 3 x 2MNK / t."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402
from hetseq_amd.ops import h3p  # noqa: E402

SHAPES = [  # name, M, N, K, ta, tb
    ("qkv fwd", 4096, 2304, 768, 0, 1), ("out fwd", 4096, 768, 768, 0, 1), ("ffn1 fwd", 4096, 3072, 768, 0, 1),
    ("ffn2 fwd", 4096, 768, 3072, 0, 1),
    ("qkv fwd half", 2048, 2304, 768, 0, 1), ("ffn2 fwd half", 2048, 768, 3072, 0, 1),
    ("qkv dgrad", 4096, 768, 2304, 0, 0), ("out dgrad", 4096, 768, 768, 0, 0), ("ffn1 dgrad", 4096, 768, 3072, 0, 0),
    ("ffn2 dgrad", 4096, 3072, 768, 0, 0),
    ("qkv wgrad", 2304, 768, 4096, 1, 0), ("out wgrad", 768, 768, 4096, 1, 0), ("ffn1 wgrad", 3072, 768, 4096, 1, 0),
    ("ffn2 wgrad", 768, 3072, 4096, 1, 0),
]


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


VARIANTS = [("h3p", lambda: None)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = []
    for name, M, N, K, ta, tb in SHAPES:
        a = torch.randn((K, M) if ta else (M, K), device=dev)
        b = torch.randn((N, K) if tb else (K, N), device=dev) * 0.05
        out = torch.empty(M, N, device=dev)
        am = (G.amax_of(a), G.amax_of(b))
        ha, hb = h3p.split(a), h3p.split(b)
        ks_opts = [s for s in (1, 2, 4, 8) if K % (32 * s) == 0 and K // s >= 256 and K // s <= 4096]
        best = {}
        for _ in range(args.rounds):
            for ks in (0, 1, 2, 4):
                if not G._hip_gemm(a, b, ta, tb, out, fp32="h3", ksplit=ks, amax=am):
                    continue
                t = timeit(lambda: G._hip_gemm(a, b, ta, tb, out, fp32="h3", ksplit=ks, amax=am))
                best[("h3", ks)] = min(best.get(("h3", ks), 1e9), t)
            for vn, setv in VARIANTS:
                setv()
                for ks in ks_opts:
                    t = timeit(lambda: h3p.gemm(ha, hb, ta, tb, out=out, ksplit=ks))
                    best[(vn, ks)] = min(best.get((vn, ks), 1e9), t)
            VARIANTS[0][1]()
        tf = lambda t: 3 * 2.0 * M * N * K / (t * 1e-6) / 1e12  # noqa: E731
        r = {"name": name, "M": M, "N": N, "K": K, "ta": ta, "tb": tb}
        for vn in ["h3"] + [v[0] for v in VARIANTS]:
            t, k = min((best[key], key[1]) for key in best if key[0] == vn)
            r[vn] = round(t, 1)
            r[vn + "_ks"] = k
            r[vn + "_tf16"] = round(tf(t))
            r[vn + "_by_ks"] = {key[1]: round(best[key], 1) for key in best if key[0] == vn}
        rows.append(r)
        print(json.dumps(r), flush=True)
    tot = {vn: round(sum(r[vn] for r in rows if "half" not in r["name"]), 1) for vn in ["h3"] + [v[0] for v in VARIANTS]}
    print(json.dumps({"layer_12_products_us": tot}))
    if args.json:
        with open(args.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
