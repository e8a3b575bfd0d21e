#!/usr/bin/env python3
"""Attention forward / backward kernel times on the BERT shapes, per fp32 product engine.

    python tools/bench_attention.py [--reps 20]

Phase 1: B=32, S=128, NH=12 (fused one-block-per-head backward); phase 2: B=8, S=512, NH=12
(dQ + dKV kernel pair).  Engines: h3 (split-fp16 products, default), x6 (split-bf16 products on the
bf16 matrix cores) and native
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
    ap.add_argument("--phases", action="store_true",
                    help="key-block backward phase clock (shader-clock stamps per block) at B=32 S=128")
    a = ap.parse_args()
    if a.phases:
        return phases()
    torch.manual_seed(0)
    for B, S, NH in [(32, 128, 12), (8, 512, 12)]:
        H = NH * 64
        qkv = torch.randn(B * S, 3 * H, device="cuda")
        bias = torch.randn(3 * H, device="cuda") * 0.1
        mask = torch.ones(B, S, dtype=torch.int64, device="cuda")
        mask[:, S - S // 8:] = 0
        row = []
        for name, mode in (("h3", 2), ("x6", 1), ("native", 0)):
            hip().set_attn_fp32_mode(mode)
            out, saved = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias)
            dout = torch.randn_like(out)
            tf = timeit(lambda: bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias), a.reps)
            tb = timeit(lambda: bert_ops.attn_bwd(qkv, mask, out, dout, saved, B, S, NH, 0.1, bias=bias), a.reps)
            row.append("%s fwd %.1f us bwd %.1f us" % (name, tf, tb))
        if S > 128:  # h3 backward staging: LDS-DMA prefetch vs per-chunk loads
            hip().set_attn_fp32_mode(2)
            out, saved = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias)
            dout = torch.randn_like(out)
            for name, on in (("dma", 1), ("loads", 0)):
                hip().set_attn_h3_dma(on)
                tb = timeit(lambda: bert_ops.attn_bwd(qkv, mask, out, dout, saved, B, S, NH, 0.1, bias=bias), a.reps)
                row.append("h3 bwd[%s] %.1f us" % (name, tb))
            hip().set_attn_h3_dma(1)
        hip().set_attn_fp32_mode(1)
        out, saved = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias)
        dout = torch.randn_like(out)
        for fam, code in (("planes", 1), ("old", 0)):  # fp32 forward kernels
            hip().set_attn_fwd_x6_planes(code)
            tf = timeit(lambda: bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias), a.reps)
            row.append("x6 fwd[%s] %.1f us" % (fam, tf))
        hip().set_attn_fwd_x6_planes(1)
        for fam, code in (("keyblock", 2), ("keyblock4", 4), ("planes", 1)):  # fp32 backward kernel families
            hip().set_attn_bwd_x6_planes(code)
            tb = timeit(lambda: bert_ops.attn_bwd(qkv, mask, out, dout, saved, B, S, NH, 0.1, bias=bias), a.reps)
            row.append("x6 bwd[%s] %.1f us" % (fam, tb))
        hip().set_attn_bwd_x6_planes(-1)
        print("B=%d S=%d NH=%d: %s" % (B, S, NH, " | ".join(row)), flush=True)


def phases():
    """Per-phase shader clocks of the key-block backward: stamp k of block b = s_memtime at point k
    (0 start, then per 64-query chunk: top, after staging barrier, after phase-A barrier; then the
    hand-off barrier and the end)."""
    torch.manual_seed(0)
    B, S, NH = 32, 128, 12
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device="cuda")
    bias = torch.randn(3 * H, device="cuda") * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device="cuda")
    hip().set_attn_fp32_mode(1)
    out, saved = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bias)
    dout = torch.randn_like(out)
    hip().set_attn_bwd_x6_planes(2)
    for _ in range(3):
        bert_ops.attn_bwd(qkv, mask, out, dout, saved, B, S, NH, 0.1, bias=bias)
    tb = torch.zeros(B * NH * 16, dtype=torch.int64, device="cuda")
    hip().set_attn_timing(tb.data_ptr())
    bert_ops.attn_bwd(qkv, mask, out, dout, saved, B, S, NH, 0.1, bias=bias)
    torch.cuda.synchronize()
    hip().set_attn_timing(0)
    t = tb.view(B * NH, 16).cpu().double()
    n = int((t[0] != 0).sum())
    t = t[:, :n]
    t0 = t[:, 0].min()
    d = t[:, 1:] - t[:, :-1]
    names = ["prologue", "chunk0 staging", "chunk0 phase A", "chunk0 phase B", "chunk1 staging", "chunk1 phase A",
             "chunk1 phase B", "hand-off + store"]
    for k in range(d.shape[1]):
        print("%-18s median %7.0f  p90 %7.0f cycles" % (names[k] if k < len(names) else k, d[:, k].median(),
                                                         d[:, k].quantile(0.9)))
    life = t[:, -1] - t[:, 0]
    print("block life median %.0f cycles; start offsets (cycles from the first block): %s" % (
        life.median(), sorted(set(int(x) // 1000 * 1000 for x in (t[:, 0] - t0).tolist()))[:12]))
    print("span first start -> last end: %.0f cycles" % (t[:, -1].max() - t0))


if __name__ == "__main__":
    main()
