#!/usr/bin/env python3
"""The h3p operand producers on the BERT-base shapes: each fp32 producer alone, with its planes
written by the producer itself (the fused *_h3p kernels), and followed by a split pass.

    python tools/bench_producers.py [--reps 30] [--json out.jsonl]

Half-batch rows (2048: the forward's two chains) and whole-batch rows (4096: the backward).
Prints median us per call."""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import bert_ops  # noqa: E402
from hetseq_amd.ops import h3p  # noqa: E402
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
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, F, NH, S = 768, 3072, 12, 128
    hip().set_attn_fp32_mode(2)
    res = []

    def rec(name, **kw):
        r = dict(name=name, **{k: round(v, 1) for k, v in kw.items()})
        res.append(r)
        print(json.dumps(r), flush=True)

    g, bt, bias = torch.randn(H, device=dev), torch.randn(H, device=dev), torch.randn(H, device=dev)
    for rows, ks in ((2048, 2), (2048, 4), (4096, 1)):
        slab = torch.randn(ks, rows, H, device=dev)
        resid = torch.randn(rows, H, device=dev)
        outs = tuple(torch.empty(rows, H, device=dev) for _ in range(2)) + tuple(
            torch.empty(rows, device=dev) for _ in range(2))
        hp = h3p.empty(rows, H, dev)
        a_in = slab if ks > 1 else slab[0]
        t0 = timeit(lambda: bert_ops.ln_fwd(a_in, g, bt, 1e-12, bias, resid, 0.1, 1, 1, 2, outs=outs), a.reps)
        tv = {}
        for _ in range(3):  # interleaved rounds (one process)
            for mode, fns in ((0, 1), (1, 1), (1, 0), (16, 1), (8, 1)):
                hip().set_ln_h3p_waves(mode)
                hip().set_ln_fwd_ns(fns)
                t = timeit(lambda: bert_ops.ln_fwd_h3p(a_in, g, bt, 1e-12, bias, resid, 0.1, 1, 2, outs, 0, hp),
                           a.reps)
                tv[mode, fns] = min(tv.get((mode, fns), 1e9), t)
        hip().set_ln_h3p_waves(1)
        hip().set_ln_fwd_ns(1)
        t2 = timeit(lambda: (bert_ops.ln_fwd(a_in, g, bt, 1e-12, bias, resid, 0.1, 1, 1, 2, outs=outs),
                             h3p.split(outs[0], out=hp)), a.reps)
        ts = timeit(lambda: h3p.split(outs[0], out=hp), a.reps)
        rec("ln_fwd rows=%d nslab=%d" % (rows, ks), fp32=t0, coop_8rows=tv[0, 1], coop_4rows=tv[1, 1],
            coop_4rows_runtime_slabs=tv[1, 0], block32_16waves=tv[16, 1], block32_8waves=tv[8, 1], then_split=t2,
            split_alone=ts)

    rows = 4096
    dy, z = torch.randn(rows, H, device=dev), torch.randn(rows, H, device=dev)
    mean, rstd = torch.randn(rows, device=dev), torch.rand(rows, device=dev) + 0.5
    acc = tuple(torch.zeros(H, device=dev) for _ in range(3))
    hp = h3p.empty(rows, H, dev)
    t0 = timeit(lambda: bert_ops.ln_bwd(dy, z, mean, rstd, g, 0.1, 1, 1, 2, True, True, acc=acc), a.reps)
    t1 = timeit(lambda: bert_ops.ln_bwd_h3p(dy, z, mean, rstd, g, 0.1, 1, 2, hp, acc=acc), a.reps)
    part32 = bert_ops._colpart_buf(rows // 32, H, dev)
    dz = torch.empty_like(dy)

    def old_bwd():  # the 32-row-block kernel (no panel record), partials only
        hip().ln_bwd_h3p(dy.data_ptr(), z.data_ptr(), mean.data_ptr(), rstd.data_ptr(), g.data_ptr(), dz.data_ptr(),
                         part32[0].data_ptr(), part32[1].data_ptr(), part32[2].data_ptr(), rows, H, 0.1, 1, 2,
                         hp.data_ptr(), hp.ps, hp.exps_ptr(), 0, torch.cuda.current_stream().cuda_stream)
    t1o = timeit(old_bwd, a.reps)

    t2 = timeit(lambda: h3p.split(bert_ops.ln_bwd(dy, z, mean, rstd, g, 0.1, 1, 1, 2, True, True, acc=acc)[1],
                                  out=hp), a.reps)
    rec("ln_bwd rows=%d" % rows, fp32=t0, fused_h3p=t1, block32_kernel_only=t1o, then_split=t2)

    for B in (16, 32):
        T = B * S
        qkv = torch.randn(T, 3 * H, device=dev)
        bq = torch.randn(3 * H, device=dev) * 0.1
        mask = torch.ones(B, S, dtype=torch.int64, device=dev)
        outs = (torch.empty(T, H, device=dev), torch.empty(B * NH * S, device=dev),
                torch.empty(B * NH * S * (S // 32), dtype=torch.int32, device=dev))
        hp = h3p.empty(T, H, dev)
        t0 = timeit(lambda: bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bq, outs=outs), a.reps)
        t1 = timeit(lambda: bert_ops.attn_fwd_h3p(qkv, mask, B, S, NH, 0.1, 1, 2, bq, outs, 0, hp), a.reps)
        t2 = timeit(lambda: (bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 1, 2, bias=bq, outs=outs),
                             h3p.split(outs[0], out=hp)), a.reps)
        rec("attn_fwd B=%d" % B, fp32=t0, fused_h3p=t1, then_split=t2)
        if B == 32:
            ctx = outs[0]
            dctx = torch.randn_like(ctx)
            hq = h3p.empty(T, 3 * H, dev)
            t0 = timeit(lambda: bert_ops.attn_bwd(qkv, mask, ctx, dctx, (outs[1], outs[2]), B, S, NH, 0.1, bias=bq),
                        a.reps)
            t1 = timeit(lambda: bert_ops.attn_bwd_h3p(qkv, mask, ctx, dctx, (outs[1], outs[2]), B, S, NH, 0.1, bq, hq),
                        a.reps)
            t2 = timeit(lambda: h3p.split(bert_ops.attn_bwd(qkv, mask, ctx, dctx, (outs[1], outs[2]), B, S, NH, 0.1,
                                                            bias=bq), out=hq), a.reps)
            tp = timeit(lambda: bert_ops.attn_bwd_h3p(qkv, mask, ctx, dctx, (outs[1], outs[2]), B, S, NH, 0.1, bq, hq,
                                                      fp32=False), a.reps)
            rec("attn_bwd B=%d" % B, fp32=t0, fused_h3p=t1, then_split=t2, planes_only=tp)
    if a.json:
        with open(a.json, "w") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
