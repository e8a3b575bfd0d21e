"""Epoch / shard / group iterators (reference: data/iterators.py:10-275).

Behaviour kept from the reference (the cross-rank "index
randomisation and assignment"):

* the global batch list is frozen once;
* epoch ``e`` visits it in the order of a legacy-NumPy shuffle seeded with
  ``seed + e`` -- the same permutation on every rank;
* rank ``r`` of ``W`` takes every W-th batch starting at ``r`` and pads its
  share with ``[]`` up to ``ceil(len / W)``, so every rank runs the same number
  of updates (the controller turns ``[]`` into a dummy ``loss * 0`` batch);
* ``state_dict`` stores (epoch, iterations_in_epoch) and resuming skips the
  batches already consumed in that epoch.

MI355X-native data path: datasets that can build a native prefetcher
(``BertH5Dataset.make_batch_stream``) are read by C++ worker threads into
pinned staging slots and copied to the GPU with ``non_blocking`` copies on a
dedicated HIP stream, event-fenced to the compute stream -- no DataLoader
worker processes and no pageable blocking copies.  Any other dataset goes
through a ``torch.utils.data.DataLoader`` over this rank's batch list.
"""
from __future__ import annotations

import itertools
import os

import numpy as np
import torch

from hetseq_amd.data import data_utils


def shard_batches(batches, num_shards, shard_id, fill_value=None):
    """Strided share ``batches[shard_id::num_shards]`` padded to ``ceil(len / num_shards)``."""
    if not 0 <= shard_id < num_shards:
        raise ValueError("shard_id must be between 0 and num_shards")
    share = list(batches[shard_id::num_shards])
    want = -(-len(batches) // num_shards)
    return share + [fill_value] * (want - len(share))


def epoch_order(batches, seed):
    """``batches`` permuted by the legacy global NumPy RNG seeded with ``seed`` (RNG state restored)."""
    out = list(batches)
    with data_utils.numpy_seed(seed):
        np.random.shuffle(out)
    return out


class CountingIterator(object):
    """Iterator over ``iterable`` that counts the items handed out (``count``), starting at ``start``."""

    def __init__(self, iterable, start=0):
        self.iterable = iterable
        self.count = start
        self.len = start + len(iterable)
        self._src = None  # started lazily on the first item (DataLoader workers fork after set_epoch)

    def __len__(self):
        return self.len

    def __iter__(self):
        return self

    def __next__(self):
        if self._src is None:
            self._src = iter(self.iterable)
        item = next(self._src)
        self.count += 1
        return item

    def has_next(self):
        return self.count < self.len

    def skip(self, num_to_skip):
        for _ in itertools.islice(self, num_to_skip):
            pass
        return self


class EpochBatchIterating(object):
    """Interface of a resumable multi-epoch batch iterator."""

    def __len__(self) -> int:
        raise NotImplementedError

    def next_epoch_itr(self, shuffle=True, fix_batches_to_gpus=False):
        raise NotImplementedError

    def end_of_epoch(self) -> bool:
        raise NotImplementedError

    @property
    def iterations_in_epoch(self) -> int:
        raise NotImplementedError

    def state_dict(self):
        raise NotImplementedError

    def load_state_dict(self, state_dict):
        raise NotImplementedError


class EpochBatchIterator(EpochBatchIterating):
    """Multi-epoch, sharded, resumable iterator over ``dataset`` with frozen batches."""

    def __init__(self, dataset, collate_fn, batch_sampler, seed=1, num_shards=1, shard_id=0, num_workers=0, epoch=0,
                 device=None):
        assert isinstance(dataset, torch.utils.data.Dataset)
        self.dataset = dataset
        self.collate_fn = collate_fn
        self.frozen_batches = tuple(batch_sampler)
        self.seed = seed
        self.num_shards = num_shards
        self.shard_id = shard_id
        self.num_workers = num_workers
        self.device = device
        self.epoch = epoch
        self.shuffle = True
        self._cur_epoch_itr = None
        self._next_epoch_itr = None  # set by load_state_dict: the resumed, partly consumed epoch
        self._supports_prefetch = getattr(dataset, "supports_prefetch", False)

    def __len__(self):
        return len(self.frozen_batches)

    @property
    def resuming(self) -> bool:
        """True between ``load_state_dict`` of a mid-epoch position and the next ``next_epoch_itr``."""
        return self._next_epoch_itr is not None

    def next_epoch_itr(self, shuffle=True, fix_batches_to_gpus=False):
        if self.resuming:
            self._cur_epoch_itr, self._next_epoch_itr = self._next_epoch_itr, None
        else:
            self.epoch += 1
            self.shuffle = shuffle
            self._cur_epoch_itr = self._open(self.epoch, shuffle, fix_batches_to_gpus=fix_batches_to_gpus)
        set_epoch = getattr(self.dataset, "set_epoch", None)
        if set_epoch is not None:
            set_epoch(self.epoch)
        return self._cur_epoch_itr

    def end_of_epoch(self) -> bool:
        return not self._cur_epoch_itr.has_next()

    @property
    def iterations_in_epoch(self):
        itr = self._cur_epoch_itr if self._cur_epoch_itr is not None else self._next_epoch_itr
        return 0 if itr is None else itr.count

    def state_dict(self):
        return {"epoch": self.epoch, "iterations_in_epoch": self.iterations_in_epoch, "shuffle": self.shuffle}

    def load_state_dict(self, state_dict):
        self.epoch = state_dict["epoch"]
        done = state_dict.get("iterations_in_epoch", 0)
        if done > 0:
            self._next_epoch_itr = self._open(self.epoch, state_dict.get("shuffle", True), offset=done)

    def epoch_batches(self, epoch, shuffle, fix_batches_to_gpus=False):
        """This rank's batch list for ``epoch`` (exposed for tests/tools)."""
        order = epoch_order(self.frozen_batches, self.seed + epoch) if shuffle and not (
            self._supports_prefetch and fix_batches_to_gpus) else list(self.frozen_batches)
        mine = shard_batches(order, self.num_shards, self.shard_id, fill_value=[])
        if self._supports_prefetch:
            self.dataset.prefetch([i for b in mine for i in b])
            if shuffle and fix_batches_to_gpus:
                mine = epoch_order(mine, self.seed + epoch + self.shard_id)
        return mine

    def _open(self, epoch, shuffle, fix_batches_to_gpus=False, offset=0):
        mine = self.epoch_batches(epoch, shuffle, fix_batches_to_gpus)
        if offset > 0 and offset >= len(mine):
            return None
        todo = mine[offset:]
        make_stream = getattr(self.dataset, "make_batch_stream", None)
        if make_stream is not None:
            src = make_stream(todo, num_threads=max(1, self.num_workers), device=self.device)
        else:
            if self.num_workers > 0:
                os.environ["PYTHONWARNINGS"] = "ignore:semaphore_tracker:UserWarning"
            src = torch.utils.data.DataLoader(self.dataset, collate_fn=self.collate_fn, batch_sampler=todo,
                                              num_workers=self.num_workers)
        return CountingIterator(src, start=offset)


class GroupedIterator(object):
    """Yields lists of ``chunk_size`` consecutive items (the last one may be shorter): update-freq groups."""

    def __init__(self, iterable, chunk_size):
        self.itr = iterable
        self.chunk_size = chunk_size
        self._len = -(-len(iterable) // chunk_size)
        self.offset = -(-getattr(iterable, "count", 0) // chunk_size)

    def __len__(self):
        return self._len

    def __iter__(self):
        return self

    def __next__(self):
        group = list(itertools.islice(self.itr, self.chunk_size))
        if not group:
            raise StopIteration
        return group


class ShardedIterator(object):
    """Iterator over this shard's strided share of ``iterable``, padded with ``fill_value``."""

    def __init__(self, iterable, num_shards, shard_id, fill_value=None):
        items = iterable if hasattr(iterable, "__getitem__") else list(iterable)
        self._items = shard_batches(items, num_shards, shard_id, fill_value)
        self._pos = iter(self._items)

    def __len__(self):
        return len(self._items)

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._pos)
