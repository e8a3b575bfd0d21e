"""The h3 attention kernels on the BERT-base shapes, repeated, for counter profiles:

    rocprofv3 --pmc ... -- python3 tools/prof_attn.py [--S 128] [--iters 30]

Forward on a half batch (the split forward's call: B 16 at S 128, B 4 at S 512), backward on the
whole batch (B 32 / 8), dropout 0.1, outputs also as h3p planes (the training step's calls)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import bert_ops  # noqa: E402
from hetseq_amd.ops import h3p  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, NH, S = 768, 12, a.S
    Bw = 32 if S == 128 else 8
    for B, bwd in ((Bw // 2, False), (Bw, True)):
        T = B * S
        qkv = torch.randn(T, 3 * H, device=dev)
        bq = torch.randn(3 * H, device=dev) * 0.1
        mask = torch.ones(B, S, dtype=torch.int64, device=dev)
        outs = (torch.empty(T, H, device=dev), torch.empty(B * NH * S, device=dev),
                torch.empty(B * NH * S * (S // 32), dtype=torch.int32, device=dev))
        hp = h3p.empty(T, H, dev)
        for _ in range(a.iters if not bwd else 1):
            bert_ops.attn_fwd_h3p(qkv, mask, B, S, NH, a.p, 1, 2, bq, outs, 0, hp)
        if bwd:
            dctx = torch.randn(T, H, device=dev)
            hq = h3p.empty(T, 3 * H, dev)
            for _ in range(a.iters):
                bert_ops.attn_bwd_h3p(qkv, mask, outs[0], dctx, (outs[1], outs[2]), B, S, NH, a.p, bq, hq, fp32=False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
