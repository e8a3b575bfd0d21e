"""Data layer: native batcher parity, iterator assignment, HDF5 shards, MNIST."""
import os

import numpy as np
import pytest
import torch

from hetseq_amd.data import data_utils, iterators


@pytest.mark.parametrize("seed", range(6))
def test_native_batcher_matches_reference_algorithm(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    lens = rng.integers(1, 60, size=n)
    idx = rng.permutation(n)
    max_tokens = int(rng.choice([None, 200, 512, 1000]) or 0) or None
    max_sent = int(rng.choice([0, 3, 8, 17])) or None
    mult = int(rng.choice([1, 2, 4, 8]))
    if max_tokens is not None:
        max_tokens = max(max_tokens, int(lens.max()))
    fn = lambda i: int(lens[i])  # noqa: E731
    ref = data_utils.batch_by_size_py(idx, fn, max_tokens, max_sent, mult)
    got = data_utils.batch_by_size(idx, fn, max_tokens, max_sent, mult)
    assert [list(map(int, b)) for b in got] == ref


def test_batcher_constant_length_fast_path():
    class DS:
        constant_num_tokens = 512

        def num_tokens(self, i):
            return 512

    ds = DS()
    got = data_utils.batch_by_size(np.arange(1000), ds.num_tokens, None, 32, 8)
    ref = data_utils.batch_by_size_py(np.arange(1000), ds.num_tokens, None, 32, 8)
    assert [list(map(int, b)) for b in got] == ref
    assert all(len(b) == 32 for b in got[:-1])


def test_batcher_raises_like_reference_assert():
    with pytest.raises(AssertionError):
        data_utils.batch_by_size(np.arange(4), lambda i: 100, 50, None, 1)


class _Toy(torch.utils.data.Dataset):
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return torch.tensor([i])

    def collater(self, s):
        return None if len(s) == 0 else torch.cat(s)


def test_sharded_assignment_golden():
    """SURVEY probe 5: 40 samples, 4 per batch, 3 ranks -> 10 batches, strided shards padded with []."""
    batches = [list(range(4 * i, 4 * i + 4)) for i in range(10)]
    per_rank = []
    for r in range(3):
        it = iterators.EpochBatchIterator(_Toy(40), _Toy(40).collater, batches, seed=19940802, num_shards=3,
                                          shard_id=r)
        per_rank.append([(b[0] // 4 if b else None) for b in it.epoch_batches(1, shuffle=True)])
    assert per_rank == [[2, 5, 0, 7], [3, 6, 1, None], [4, 8, 9, None]]
    # all batches used exactly once
    flat = sorted(x for r in per_rank for x in r if x is not None)
    assert flat == list(range(10))


def test_epoch_iterator_resume_offset():
    batches = [list(range(4 * i, 4 * i + 4)) for i in range(10)]
    it = iterators.EpochBatchIterator(_Toy(40), _Toy(40).collater, batches, seed=19940802, num_shards=3, shard_id=0)
    e = it.next_epoch_itr()
    next(e), next(e)
    st = it.state_dict()
    assert st["epoch"] == 1 and st["iterations_in_epoch"] == 2
    it2 = iterators.EpochBatchIterator(_Toy(40), _Toy(40).collater, batches, seed=19940802, num_shards=3,
                                       shard_id=0)
    it2.load_state_dict(st)
    rest = [b.tolist() for b in it2.next_epoch_itr()]
    assert [r[0] // 4 for r in rest] == [0, 7]


def test_grouped_iterator():
    g = iterators.GroupedIterator(iterators.CountingIterator(list(range(7))), 3)
    assert len(g) == 3
    assert list(g) == [[0, 1, 2], [3, 4, 5], [6]]


def _oracle_labels(pos, ids, S, max_pred=512):
    lab = np.full(S, -1, np.int64)
    k = len(pos)
    z = np.nonzero(pos == 0)[0]
    if len(z):
        k = z[0]
    k = min(k, max_pred)
    lab[pos[:k]] = ids[:k]
    return lab


def test_h5_shards_roundtrip_and_labels(tmp_path):
    from hetseq_amd.data.bert_dataset import BertH5Dataset, ConBertH5Dataset
    from hetseq_amd.data.synthetic import make_bert_arrays, write_bert_shards

    paths = write_bert_shards(str(tmp_path), num_shards=2, per_shard=50, seq_len=32, max_pred=6, vocab_size=500,
                              seed=3, gzip_level=1)
    ds = ConBertH5Dataset([BertH5Dataset(p) for p in paths])
    assert len(ds) == 100 and ds.seq_len == 32 and ds.num_pred == 6
    ids, mask, seg, pos, mids, nsp = make_bert_arrays(50, 32, 6, 500, seed=3 * 1000 + 1)
    s = ds[57]  # shard 1, row 7
    assert s[0].tolist() == ids[7].tolist()
    assert s[1].tolist() == seg[7].tolist() and s[2].tolist() == mask[7].tolist()
    assert s[3].tolist() == _oracle_labels(pos[7], mids[7], 32).tolist()
    assert int(s[4]) == int(nsp[7])
    # collated native gather == per-sample path, across the shard boundary
    idx = [48, 49, 50, 51, 3]
    b = ds.read_batch(idx)
    ref = ds.collater([ds[i] for i in idx])
    for x, y in zip(b, ref):
        assert torch.equal(x, y)


def test_native_prefetch_stream_cpu(tmp_path):
    from hetseq_amd.data.bert_dataset import BertH5Dataset, ConBertH5Dataset
    from hetseq_amd.data.synthetic import write_bert_shards

    paths = write_bert_shards(str(tmp_path), num_shards=3, per_shard=40, seq_len=16, max_pred=4, vocab_size=300)
    ds = ConBertH5Dataset([BertH5Dataset(p) for p in paths])
    batches = data_utils.batch_by_size(ds.ordered_indices(), ds.num_tokens, None, 7, 1)
    it = iterators.EpochBatchIterator(ds, ds.collater, batches, seed=5, num_shards=2, shard_id=1, num_workers=3)
    got = list(it.next_epoch_itr())
    want = it.epoch_batches(1, True)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        if len(w) == 0:
            assert g is None
            continue
        ref = ds.collater([ds[int(i)] for i in w])
        for x, y in zip(g, ref):
            assert torch.equal(x, y)


def test_mnist_dataset_transform(tmp_path):
    from hetseq_amd.data.mnist_dataset import MNISTDataset, find_split_file
    from hetseq_amd.data.synthetic import write_mnist

    write_mnist(str(tmp_path), 20, 10)
    f = find_split_file(str(tmp_path), "train")
    ds = MNISTDataset(f)
    img, y = ds[3]
    raw, labels = torch.load(f, weights_only=True)
    ref = (raw[3].float() / 255.0 - 0.1307) / 0.3081
    assert img.shape == (1, 28, 28) and torch.allclose(img[0], ref) and y == int(labels[3])
    x, t = ds.collater([ds[0], ds[1]])
    assert x.shape == (2, 1, 28, 28) and t.dtype == torch.int64


def test_synthetic_corpus_cli(tmp_path):
    """python -m hetseq_amd.data.synthetic produces a corpus the BERT task loads."""
    from hetseq_amd.data.bert_dataset import BertH5Dataset
    from hetseq_amd.data.synthetic import main

    main([str(tmp_path), "--shards", "2", "--per-shard", "40", "--vocab-size", "500"])
    files = sorted(os.listdir(tmp_path / "data"))
    assert sum("train" in f for f in files) == 2 and sum("test" in f for f in files) == 1
    ds = BertH5Dataset(str(tmp_path / "data" / [f for f in files if "train" in f][0]), 20)
    assert len(ds) == 40
    assert (tmp_path / "vocab.txt").exists() and (tmp_path / "bert_config.json").exists()


def test_counting_and_sharded_iterators():
    c = iterators.CountingIterator(list(range(10)), start=0)
    assert next(c) == 0 and c.count == 1 and c.has_next()
    c.skip(3)
    assert c.count == 4 and next(c) == 4
    assert list(c) == [5, 6, 7, 8, 9] and not c.has_next() and len(c) == 10
    assert list(iterators.ShardedIterator(range(7), 3, 2, fill_value=-1)) == [2, 5, -1]
    assert list(iterators.ShardedIterator((x for x in range(7)), 3, 0)) == [0, 3, 6]
    assert len(iterators.ShardedIterator(range(7), 3, 1)) == 3
    with pytest.raises(ValueError):
        iterators.ShardedIterator(range(7), 3, 3)
