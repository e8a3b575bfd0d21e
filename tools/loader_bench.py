#!/usr/bin/env python3
"""Input-pipeline throughput: iterate the native HDF5 batch stream alone (no model).

usage: python tools/loader_bench.py [--batches 50] [--workers 2] [--device cuda]
"""
import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=50)
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--bsz", type=int, default=32)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    from hetseq_amd.data import data_utils, iterators
    from hetseq_amd.data.bert_dataset import BertH5Dataset, ConBertH5Dataset
    from hetseq_amd.data.synthetic import write_bert_shards

    d = tempfile.mkdtemp()
    write_bert_shards(d, num_shards=2, per_shard=a.batches * a.bsz, seq_len=128, max_pred=20, vocab_size=30522,
                      seed=1, split="train")
    files = sorted(os.path.join(d, f) for f in os.listdir(d))
    ds = ConBertH5Dataset([BertH5Dataset(f, 20) for f in files])
    itr = iterators.EpochBatchIterator(ds, ds.collater, data_utils.batch_by_size(
        ds.ordered_indices(), ds.num_tokens, max_tokens=None, max_sentences=a.bsz), seed=1,
        num_workers=a.workers, device=torch.device(a.device))
    t0 = time.perf_counter()
    n = 0
    for s in itr.next_epoch_itr(shuffle=True):
        n += 1
    if a.device == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("%d batches in %.3f s: %.3f ms/batch" % (n, dt, dt / n * 1e3))


if __name__ == "__main__":
    main()
