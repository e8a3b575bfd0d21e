#!/usr/bin/env python3
"""Attention forward / backward kernel times on the BERT shapes, per fp32 product engine.

    python tools/bench_attention.py [--reps 20]

Phase 1: B=32, S=128, NH=12; phase 2: B=8, S=512, NH=12.  Engines: h3 (split-fp16 products, default) and native
(exact-fp32 v_mfma_f32_32x32x2_f32); dropout 0.1 as in training.  Prints median us per call.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import bert_ops  # noqa: E402
from hetseq_amd.ops._C import hip  # noqa: E402


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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    for B, S, NH in [(32, 128, 12), (8, 512, 12)]:
        H = NH * 64
        qkv = torch.randn(B * S, 3 * H, device="cuda")
        bias = torch.randn(3 * H, device="cuda") * 0.1
        mask = torch.ones(B, S, dtype=torch.int64, device="cuda")
        mask[:, S - S // 8:] = 0
        row = []
        for name, mode in (("h3", 2), ("native", 0)):
            hip().set_attn_fp32_mode(mode)
            out, saved = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias)
            dout = torch.randn_like(out)
            tf = timeit(lambda: bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias), a.reps)
            tb = timeit(lambda: bert_ops.attn_bwd(qkv, mask, out, dout, saved, B, S, NH, 0.1, bias=bias), a.reps)
            row.append("%s fwd %.1f us bwd %.1f us" % (name, tf, tb))
        print("B=%d S=%d NH=%d: %s" % (B, S, NH, " | ".join(row)), flush=True)


if __name__ == "__main__":
    main()
