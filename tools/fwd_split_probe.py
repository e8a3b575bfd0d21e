#!/usr/bin/env python3
"""Probe: 12 BERT-base encoder layer forwards (fp32 fused path, no autograd) on one stream with the
whole batch vs the batch split in two halves run as independent chains on two streams -- how much
of the forward's GEMM wave-quantisation tails the other half's work fills.

    python tools/fwd_split_probe.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.models.bert import BertConfig, BertForPreTraining  # noqa: E402
from hetseq_amd.ops import bert_ops  # noqa: E402
from hetseq_amd.runtime import streams  # noqa: E402
from hetseq_amd.runtime.flat import FlatParamStore  # noqa: E402


def main():
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=30522, hidden_size=768, num_hidden_layers=12,
                     num_attention_heads=12, intermediate_size=3072)
    model = BertForPreTraining(cfg).cuda()
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    layers = model.bert.encoder.layer
    Ws = [l._weights() for l in layers]
    B, S, NH = 32, 128, 12
    x = torch.randn(B * S, 768, device="cuda")
    mask = torch.ones(B, S, dtype=torch.int64, device="cuda")
    seeds = ((1, 0), (1, 256), (1, 512))

    def run(xx, mm, b):
        c = (b, S, NH, 0.1, 0.1, 1e-12, seeds)
        h = xx
        for W in Ws:
            h, _ = bert_ops._layer_forward(h, mm, W, c, save=True)
        return h

    s2 = torch.cuda.Stream()

    def full():
        run(x, mask, B)

    def split():  # layer by layer, half 0 on the current stream, half 1 on s2 (timing only: the
        # two chains share the split-K slab, so the numbers they compute are not meaningful)
        cur = torch.cuda.current_stream()
        s2.wait_stream(cur)
        half = B * S // 2
        c = (B // 2, S, NH, 0.1, 0.1, 1e-12, seeds)
        h0, h1 = x[:half], x[half:]
        for W in Ws:
            h0, _ = bert_ops._layer_forward(h0, mask[:B // 2], W, c, save=True)
            with torch.cuda.stream(s2):
                h1, _ = bert_ops._layer_forward(h1, mask[B // 2:], W, c, save=True)
        cur.wait_stream(s2)

    s3, s4 = torch.cuda.Stream(), torch.cuda.Stream()

    def split4():  # four quarter-batch chains on four streams
        cur = torch.cuda.current_stream()
        sts = [cur, s2, s3, s4]
        for st in sts[1:]:
            st.wait_stream(cur)
        q, qb = B * S // 4, B // 4
        c = (qb, S, NH, 0.1, 0.1, 1e-12, seeds)
        hs = [x[i * q:(i + 1) * q] for i in range(4)]
        for W in Ws:
            for i in range(4):
                with torch.cuda.stream(sts[i]):
                    hs[i], _ = bert_ops._layer_forward(hs[i], mask[i * qb:(i + 1) * qb], W, c, save=True)
        for st in sts[1:]:
            cur.wait_stream(st)

    def half_only():
        run(x[:B * S // 2], mask[:B // 2], B // 2)

    bert_ops._FWD_SPLIT = False  # the probe does its own splitting
    for fn in (full, split, split4, half_only):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    res = {}
    for rep in range(6):
        for name, fn in (("full", full), ("split2", split), ("split4", split4), ("one_half", half_only)):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            res.setdefault(name, []).append(s.elapsed_time(e))
    for k, v in res.items():
        print("%-9s median %.3f ms  (%s)" % (k, statistics.median(v), " ".join("%.3f" % t for t in v)))


if __name__ == "__main__":
    main()
