"""Isolated timing of the BERT-base fp32 products: the in-kernel-split h3 engine (gemm.hip, NT=4,
per-tensor scales) against the h3p engine (gemm_h3p.hip, pre-split block-scaled planes).

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
        best_old, best_new, best_ring = {}, {}, {}
        hip = __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip()
        for _ in range(args.rounds):
            hip.set_h3p_variant(1)
            for ks in ks_opts:
                t = timeit(lambda: h3p.gemm(ha, hb, ta, tb, out=out, ksplit=ks))
                best_ring[ks] = min(best_ring.get(ks, 1e9), t)
            hip.set_h3p_variant(0)
            for ks in (0, 1, 2, 4):
                if not G._hip_gemm(a, b, ta, tb, out, fp32="h3", ksplit=ks, amax=am):
                    continue
                t = timeit(lambda: G._hip_gemm(a, b, ta, tb, out, fp32="h3", ksplit=ks, amax=am))
                best_old[ks] = min(best_old.get(ks, 1e9), t)
            for ks in ks_opts:
                t = timeit(lambda: h3p.gemm(ha, hb, ta, tb, out=out, ksplit=ks))
                best_new[ks] = min(best_new.get(ks, 1e9), t)
        to, ko = min((v, k) for k, v in best_old.items())
        tn, kn = min((v, k) for k, v in best_new.items())
        tr, kr = min((v, k) for k, v in best_ring.items())
        tf = lambda t: 3 * 2.0 * M * N * K / (t * 1e-6) / 1e12  # noqa: E731
        r = {"name": name, "M": M, "N": N, "K": K, "ta": ta, "tb": tb, "h3_us": round(to, 1), "h3_ks": ko,
             "h3p_us": round(tn, 1), "h3p_ks": kn, "h3_tf16": round(tf(to)), "h3p_tf16": round(tf(tn)),
             "speedup": round(to / tn, 3), "h3p_by_ks": {k: round(v, 1) for k, v in best_new.items()},
             "ring_us": round(tr, 1), "ring_ks": kr, "ring_tf16": round(tf(tr)), "ring_speedup": round(to / tr, 3),
             "ring_by_ks": {k: round(v, 1) for k, v in best_ring.items()}}
        rows.append(r)
        print(json.dumps(r), flush=True)
    tot_o = sum(r["h3_us"] for r in rows if "half" not in r["name"])
    tot_n = sum(r["h3p_us"] for r in rows if "half" not in r["name"])
    tot_r = sum(r["ring_us"] for r in rows if "half" not in r["name"])
    print(json.dumps({"layer_12_products_h3_us": round(tot_o, 1), "h3p_us": round(tot_n, 1),
                      "speedup": round(tot_o / tot_n, 3), "ring_us": round(tot_r, 1),
                      "ring_speedup": round(tot_o / tot_r, 3)}))
    if args.json:
        with open(args.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
