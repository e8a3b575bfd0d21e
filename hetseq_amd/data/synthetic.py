"""Synthetic data generators (there is no network for real corpora).

* ``write_bert_shards`` writes NVIDIA-format BERT pre-training HDF5 shards
  (the reference's input format, data/h5pyDataset.py:16-17) through the
  native libhdf5 writer: int32 input_ids / masked_lm_positions /
  masked_lm_ids, int8 input_mask / segment_ids / next_sentence_labels,
  optional gzip.  Each sequence has a random real length, [CLS]/[SEP]
  structure, two segments and up to ``max_pred`` sorted masked positions
  (0-padded, like create_pretraining_data.py).
* ``write_vocab`` / ``write_bert_config`` produce the dictionary and model
  JSON the BERT task expects.
* ``write_mnist`` writes ``MNIST/processed/{training,test}.pt`` tuples.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

BERT_BASE = dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_act="gelu", hidden_dropout_prob=0.1,
                 attention_probs_dropout_prob=0.1, max_position_embeddings=512, type_vocab_size=2,
                 initializer_range=0.02)


def make_bert_arrays(n, seq_len=128, max_pred=20, vocab_size=30522, seed=0, full_length=False):
    rng = np.random.default_rng(seed)
    ids = np.zeros((n, seq_len), np.int32)
    mask = np.zeros((n, seq_len), np.int8)
    seg = np.zeros((n, seq_len), np.int8)
    pos = np.zeros((n, max_pred), np.int32)
    mids = np.zeros((n, max_pred), np.int32)
    nsp = rng.integers(0, 2, size=n).astype(np.int8)
    lo = 999 if vocab_size > 1000 else 5
    for i in range(n):
        L = seq_len if full_length else int(rng.integers(max(8, seq_len // 2), seq_len + 1))
        toks = rng.integers(lo, vocab_size, size=L).astype(np.int32)
        toks[0] = 101 % vocab_size
        cut = int(rng.integers(2, L - 2))
        toks[cut] = 102 % vocab_size
        toks[L - 1] = 102 % vocab_size
        ids[i, :L] = toks
        mask[i, :L] = 1
        seg[i, cut + 1 : L] = 1
        k = min(max_pred, max(1, int(round(0.15 * L))))
        cand = np.setdiff1d(np.arange(1, L), [cut, L - 1])
        p = np.sort(rng.choice(cand, size=min(k, len(cand)), replace=False)).astype(np.int32)
        pos[i, : len(p)] = p
        mids[i, : len(p)] = toks[p]
        ids[i, p] = 103 % vocab_size  # [MASK]
    return ids, mask, seg, pos, mids, nsp


def write_bert_shards(out_dir, num_shards=2, per_shard=256, seq_len=128, max_pred=20, vocab_size=30522, seed=0,
                      split="train", gzip_level=0, full_length=False):
    from hetseq_amd.ops._C import h5

    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for s in range(num_shards):
        ids, mask, seg, pos, mids, nsp = make_bert_arrays(per_shard, seq_len, max_pred, vocab_size, seed * 1000 + s,
                                                          full_length=full_length)
        path = os.path.join(out_dir, "synthetic_seq{}_{}_{:04d}.hdf5".format(seq_len, split, s))
        h5().write_shard(path, ids, mask, seg, pos, mids, nsp, gzip_level)
        paths.append(path)
    return paths


def write_vocab(path, vocab_size=30522):
    with open(path, "w", encoding="utf-8") as f:
        specials = ["[PAD]"] + ["[unused%d]" % i for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
        for i in range(vocab_size):
            f.write((specials[i] if i < len(specials) else "tok%d" % i) + "\n")
    return path


def write_bert_config(path, **overrides):
    cfg = dict(BERT_BASE)
    cfg.update(overrides)
    with open(path, "w") as f:
        json.dump(cfg, f, indent=2)
    return path


def write_mnist(root, n_train=512, n_test=128, seed=0):
    g = torch.Generator().manual_seed(seed)
    d = os.path.join(root, "MNIST", "processed")
    os.makedirs(d, exist_ok=True)
    for name, n in (("training.pt", n_train), ("test.pt", n_test)):
        labels = torch.randint(0, 10, (n,), generator=g)
        images = torch.randint(0, 60, (n, 28, 28), generator=g, dtype=torch.int64)
        # draw a crude class-dependent pattern so the task is learnable
        for c in range(10):
            sel = labels == c
            images[sel, 2 + 2 * c : 6 + 2 * c, 4:24] += 180
        torch.save((images.clamp(0, 255).to(torch.uint8), labels), os.path.join(d, name))
    return root


def main(argv=None):
    """``python -m hetseq_amd.data.synthetic OUT_DIR``: a ready-to-train synthetic BERT corpus
    (train/test shards, vocab.txt, bert_config.json) or MNIST tensors (``--mnist``)."""
    import argparse

    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("out_dir")
    ap.add_argument("--mnist", action="store_true", help="write MNIST/processed/{training,test}.pt instead")
    ap.add_argument("--shards", type=int, default=4)
    ap.add_argument("--per-shard", type=int, default=4096, help="sequences per shard")
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--max-pred", type=int, default=20, help="20 for phase 1 (seq 128), 80 for phase 2 (seq 512)")
    ap.add_argument("--vocab-size", type=int, default=30522)
    ap.add_argument("--gzip", type=int, default=0, help="gzip level of the HDF5 datasets (0 = contiguous)")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    if a.mnist:
        write_mnist(a.out_dir, seed=a.seed)
        print("| wrote %s/MNIST/processed" % a.out_dir)
        return
    data = os.path.join(a.out_dir, "data")
    for split, n in (("train", a.shards), ("test", 1)):
        write_bert_shards(data, num_shards=n, per_shard=a.per_shard, seq_len=a.seq_len, max_pred=a.max_pred,
                          vocab_size=a.vocab_size, seed=a.seed + (0 if split == "train" else 7919), split=split,
                          gzip_level=a.gzip)
    write_vocab(os.path.join(a.out_dir, "vocab.txt"), a.vocab_size)
    write_bert_config(os.path.join(a.out_dir, "bert_config.json"), vocab_size=a.vocab_size)
    print("| wrote %s: --data %s --dict %s --config_file %s" % (a.out_dir, data, os.path.join(a.out_dir, "vocab.txt"),
                                                             os.path.join(a.out_dir, "bert_config.json")))


if __name__ == "__main__":
    main()
