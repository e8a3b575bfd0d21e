"""Precision census of the fp32 split-fp16 GEMM engines on real BERT-base training tensors.

    python tools/h3p_census.py [--steps 200] [--every 20] [--out profiles/r5_h3_census.md]

Trains BERT-base (phase 1: seq 128, 32 sequences, 20 masked positions each, dropout ON, fused Adam)
on synthetic batches and, every ``--every`` updates, records for each GEMM call site and operand the
share of nonzero elements below the precision window of their scale (|x * 2^e| < 2^-3: fewer than
22 significant bits kept) and those elements' share of the operand's |x| mass -- once with the h3p
engine (exponent per 32 x 32 block) and once with the h3 engine (one exponent per tensor) on the same
weights and batches.  Reference: the fp32 GEMMs of bert_modeling.py:352-354, 166-172, 547."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--every", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from argparse import Namespace

    from hetseq_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops import h3p

    # the Python layer (the same kernels and arguments as the native layer program, which is bitwise
    # equal to it: tests/test_layer_prog_gpu.py) -- its products pass through h3p.gemm, where the
    # census records them
    bert_ops.LAYER_PROG = False
    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.runtime import rng
    from hetseq_amd.runtime.flat import FlatParamStore

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=30522)
    model = BertForPreTraining(cfg).to(dev)
    model.train()  # dropout on
    model.max_predictions_per_seq = 20
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    opt = _Adam(Namespace(lr=[1e-4], adam_betas="(0.9,0.999)", adam_eps=1e-6, weight_decay=0.01),
                list(model.parameters()), store)
    B, S, P = a.batch, 128, 20
    g = torch.Generator(device="cpu").manual_seed(1)

    def batch():
        ids = torch.randint(0, cfg.vocab_size, (B, S), generator=g)
        tt = (torch.arange(S) > S // 2).long().expand(B, S).contiguous()
        mask = torch.ones(B, S, dtype=torch.long)
        labels = torch.full((B, S), -1, dtype=torch.long)
        for b in range(B):
            pos = torch.randperm(S - 2, generator=g)[:P] + 1
            labels[b, pos] = torch.randint(0, cfg.vocab_size, (P,), generator=g)
        nsp = torch.randint(0, 2, (B,), generator=g)
        return tuple(t.to(dev) for t in (ids, tt, mask, labels, nsp))

    totals = {}
    t0 = time.time()
    for step in range(a.steps):
        bt = batch()
        sample = (step + 1) % a.every == 0
        for eng in (("h3", "h3p") if sample else ("h3p",)):  # (the update uses h3p's gradients)
            rng.set_seed(1000 + step)  # the same dropout masks for both engines
            G.set_fp32_mode(eng)
            if sample:
                h3p.census_start()
            opt.zero_grad()
            loss = model(*bt)
            loss.backward()
            if sample:
                for k, v in h3p.census_stop().items():
                    key = (eng,) + (k if k[0] != "h3" else k[1:])
                    acc = totals.setdefault(key, [0, 0, 0.0, 0.0, 0])
                    for i in range(5):
                        acc[i] += v[i]
        G.set_fp32_mode("h3p")
        opt.clip_grad_norm(1.0)
        opt.step()
        if step % 20 == 0:
            print("step %d loss %.4f (%.0f s)" % (step, loss.item(), time.time() - t0), flush=True)
    lines = ["# fp32 split-fp16 GEMM precision census, BERT-base phase 1 (%d updates, dropout on, every %d sampled)"
             % (a.steps, a.every), "",
             "Share of nonzero operand elements below their scale's 2^18 window (|x * 2^e| < 2^-3: fewer than 22 "
             "significant bits), and their share of the operand's |x| mass, per call site; h3p = one exponent "
             "per 32 x 32 block, h3 = one per tensor (same weights, same batches).", "",
             "| engine | site | operand | calls | elements below window | |x| mass below window |",
             "|---|---|---|---|---|---|"]
    for key in sorted(totals, key=lambda k: (k[0], str(k[1:]))):
        nz, out, mo, mt, n = totals[key]
        lines.append("| %s | %s | %s | %d | %.3g | %.3g |" % (key[0], " ".join(str(x) for x in key[1:-1]), key[-1], n,
                                                               out / max(nz, 1), mo / max(mt, 1e-300)))
    # the same h3p tensors under one exponent per tensor ("A/tensor", "B/tensor" rows): per site, the
    # per-block count must not exceed the per-tensor one (a producer writing wrong exponents would)
    viol = []
    for key in totals:
        if key[0] == "h3p" and not str(key[-1]).endswith("/tensor"):
            tk = key[:-1] + (key[-1] + "/tensor",)
            if tk in totals and totals[key][1] > totals[tk][1]:
                viol.append(" ".join(str(x) for x in key[1:]))
    lines += ["", "Same-tensor check (h3p operands, per-block vs per-tensor window on identical values): %s"
              % ("per-block <= per-tensor at every site" if not viol else "VIOLATED at: " + "; ".join(viol))]
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
