"""The h3 attention kernels alone on the BERT-base shapes (CUDA-event timing, best of rounds):
forward on a half batch (the split forward's call: B 16 at S 128, B 4 at S 512), backward on the whole
batch, outputs also as h3p planes (the training step's calls), dropout 0.1 and 0 (the forward's share
spent on the Philox keep bits).

    python tools/bench_attn.py [--rounds 3]   (HS_AB_ROOT: time another build of the package)"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.environ.get("HS_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import bert_ops  # noqa: E402
from hetseq_amd.ops import h3p  # noqa: E402


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, NH = 768, 12
    for S, Bw in ((128, 32), (512, 8)):
        runs = {}
        for p in (0.1, 0.0):
            for B, bwd in ((Bw // 2, False), (Bw, True)):
                T = B * S
                qkv = torch.randn(T, 3 * H, device=dev)
                bq = torch.randn(3 * H, device=dev) * 0.1
                mask = torch.ones(B, S, dtype=torch.int64, device=dev)
                mask[:, S - S // 8:] = 0
                outs = (torch.empty(T, H, device=dev), torch.empty(B * NH * S, device=dev),
                        torch.empty(B * NH * S * (S // 32), dtype=torch.int32, device=dev))
                hp = h3p.empty(T, H, dev)
                fwd = (lambda qkv, mask, B, p, bq, outs, hp:
                       lambda: bert_ops.attn_fwd_h3p(qkv, mask, B, S, NH, p, 1, 2, bq, outs, 0, hp))(
                           qkv, mask, B, p, bq, outs, hp)
                if not bwd:
                    runs["fwd B%d p%g" % (B, p)] = fwd
                else:
                    fwd()
                    dctx = torch.randn(T, H, device=dev)
                    hq = h3p.empty(T, 3 * H, dev)
                    runs["bwd B%d p%g" % (B, p)] = (lambda qkv, mask, outs, dctx, B, p, bq, hq:
                                                   lambda: bert_ops.attn_bwd_h3p(qkv, mask, outs[0], dctx,
                                                                                 (outs[1], outs[2]), B, S, NH, p,
                                                                                 bq, hq, fp32=False))(
                        qkv, mask, outs, dctx, B, p, bq, hq)
        from hetseq_amd.ops._C import hip
        bwd = [k for k in runs if k.startswith("bwd")]
        for role, tag in ((1, "dkv only"), (2, "dq only")):  # (diagnostic: one backward role's blocks)
            for k in bwd:
                runs["%s %s" % (k, tag)] = (lambda fn, r: lambda: (hip().set_attn_h3_variant(-1, r), fn(),
                                                                    hip().set_attn_h3_variant(-1, 3)))(runs[k], role)
        if "ds" in __import__("inspect").signature(bert_ops.attn_bwd_h3p).parameters:
            for p_ in (0.1, 0.0):  # dQ from the stored dS (the layer program's path)
                B = Bw
                T = B * S
                qkv = torch.randn(T, 3 * H, device=dev)
                bq = torch.randn(3 * H, device=dev) * 0.1
                mask = torch.ones(B, S, dtype=torch.int64, device=dev)
                outs = (torch.empty(T, H, device=dev), torch.empty(B * NH * S, device=dev),
                        torch.empty(B * NH * S * (S // 32), dtype=torch.int32, device=dev))
                bert_ops.attn_fwd_h3p(qkv, mask, B, S, NH, p_, 1, 2, bq, outs, 0, h3p.empty(T, H, dev))
                dctx, hq = torch.randn(T, H, device=dev), h3p.empty(T, 3 * H, dev)
                runs["bwd B%d p%g ds" % (B, p_)] = (lambda qkv, mask, outs, dctx, B, p_, bq, hq:
                                                    lambda: bert_ops.attn_bwd_h3p(qkv, mask, outs[0], dctx,
                                                                                  (outs[1], outs[2]), B, S, NH, p_,
                                                                                  bq, hq, fp32=False, ds=True))(
                    qkv, mask, outs, dctx, B, p_, bq, hq)
        best = {}
        for _ in range(a.rounds):
            for k, fn in runs.items():
                best[k] = min(best.get(k, 1e9), timeit(fn))
        print(json.dumps({"S": S, **{k: round(v, 1) for k, v in best.items()}}), flush=True)


if __name__ == "__main__":
    main()
