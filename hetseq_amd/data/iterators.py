"""Epoch / shard / group iterators (reference: data/iterators.py:10-275).

Index randomisation and assignment across ranks are kept exactly (the heart
of HetSeq): the frozen global batch list is shuffled per epoch
with ``seed + epoch`` (identical on every rank), sharded STRIDED
(``batches[shard_id::num_shards]``), and short shards are padded with ``[]``
so that every rank runs the same number of updates; ``state_dict`` /
``load_state_dict`` fast-forward inside an epoch.

MI355X-native data path: when the dataset can build a native prefetcher
(``BertH5Dataset``), batches are read by C++ worker threads straight into
pinned staging slots and copied to the GPU with ``non_blocking`` copies on a
dedicated HIP stream, event-fenced to the compute stream -- no DataLoader
worker processes and no pageable blocking copies.  Other datasets use a
``torch.utils.data.DataLoader`` exactly like the reference.
"""
from __future__ import annotations

import itertools
import math
import os

import numpy as np
import torch

from hetseq_amd.data import data_utils


class CountingIterator(object):
    """Wrapper around an iterable that maintains the iteration count."""

    def __init__(self, iterable, start=0):
        self.iterable = iterable
        self.count = start
        self.itr = iter(self)
        self.len = start + len(iterable)

    def __len__(self):
        return self.len

    def __iter__(self):
        for x in self.iterable:
            self.count += 1
            yield x

    def __next__(self):
        return next(self.itr)

    def has_next(self):
        return self.count < len(self)

    def skip(self, num_to_skip):
        next(itertools.islice(self.itr, num_to_skip, num_to_skip), None)
        return self


class EpochBatchIterating(object):
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
    """A multi-epoch, sharded, resumable iterator over a dataset."""

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
        self._next_epoch_itr = None
        self._supports_prefetch = getattr(dataset, "supports_prefetch", False)

    def __len__(self):
        return len(self.frozen_batches)

    def next_epoch_itr(self, shuffle=True, fix_batches_to_gpus=False):
        if self._next_epoch_itr is not None:
            self._cur_epoch_itr = self._next_epoch_itr
            self._next_epoch_itr = None
        else:
            self.epoch += 1
            self.shuffle = shuffle
            self._cur_epoch_itr = self._get_iterator_for_epoch(self.epoch, shuffle,
                                                               fix_batches_to_gpus=fix_batches_to_gpus)
        if hasattr(self.dataset, "set_epoch"):
            self.dataset.set_epoch(self.epoch)
        return self._cur_epoch_itr

    def end_of_epoch(self) -> bool:
        return not self._cur_epoch_itr.has_next()

    @property
    def iterations_in_epoch(self):
        if self._cur_epoch_itr is not None:
            return self._cur_epoch_itr.count
        elif self._next_epoch_itr is not None:
            return self._next_epoch_itr.count
        return 0

    def state_dict(self):
        return {"epoch": self.epoch, "iterations_in_epoch": self.iterations_in_epoch, "shuffle": self.shuffle}

    def load_state_dict(self, state_dict):
        self.epoch = state_dict["epoch"]
        itr_pos = state_dict.get("iterations_in_epoch", 0)
        if itr_pos > 0:
            self._next_epoch_itr = self._get_iterator_for_epoch(self.epoch, shuffle=state_dict.get("shuffle", True),
                                                                offset=itr_pos)

    def epoch_batches(self, epoch, shuffle, fix_batches_to_gpus=False):
        """This rank's batch list for ``epoch`` (exposed for tests/tools)."""

        def shuffle_batches(batches, seed):
            with data_utils.numpy_seed(seed):
                np.random.shuffle(batches)
            return batches

        if self._supports_prefetch:
            batches = self.frozen_batches
            if shuffle and not fix_batches_to_gpus:
                batches = shuffle_batches(list(batches), self.seed + epoch)
            batches = list(ShardedIterator(batches, self.num_shards, self.shard_id, fill_value=[]))
            self.dataset.prefetch([i for s in batches for i in s])
            if shuffle and fix_batches_to_gpus:
                batches = shuffle_batches(batches, self.seed + epoch + self.shard_id)
        else:
            if shuffle:
                batches = shuffle_batches(list(self.frozen_batches), self.seed + epoch)
            else:
                batches = self.frozen_batches
            batches = list(ShardedIterator(batches, self.num_shards, self.shard_id, fill_value=[]))
        return batches

    def _get_iterator_for_epoch(self, epoch, shuffle, fix_batches_to_gpus=False, offset=0):
        batches = self.epoch_batches(epoch, shuffle, fix_batches_to_gpus)
        if offset > 0 and offset >= len(batches):
            return None
        remaining = batches[offset:]
        maker = getattr(self.dataset, "make_batch_stream", None)
        if maker is not None:
            stream = maker(remaining, num_threads=max(1, self.num_workers), device=self.device)
            return CountingIterator(stream, start=offset)
        if self.num_workers > 0:
            os.environ["PYTHONWARNINGS"] = "ignore:semaphore_tracker:UserWarning"
        return CountingIterator(
            torch.utils.data.DataLoader(self.dataset, collate_fn=self.collate_fn, batch_sampler=remaining,
                                        num_workers=self.num_workers),
            start=offset,
        )


class GroupedIterator(object):
    """Wrapper around an iterable that returns groups (chunks) of items."""

    def __init__(self, iterable, chunk_size):
        self._len = int(math.ceil(len(iterable) / float(chunk_size)))
        self.offset = int(math.ceil(getattr(iterable, "count", 0) / float(chunk_size)))
        self.itr = iterable
        self.chunk_size = chunk_size

    def __len__(self):
        return self._len

    def __iter__(self):
        return self

    def __next__(self):
        chunk = []
        try:
            for _ in range(self.chunk_size):
                chunk.append(next(self.itr))
        except StopIteration as e:
            if len(chunk) == 0:
                raise e
        return chunk


class ShardedIterator(object):
    """A sharded wrapper around an iterable, padded to length."""

    def __init__(self, iterable, num_shards, shard_id, fill_value=None):
        if shard_id < 0 or shard_id >= num_shards:
            raise ValueError("shard_id must be between 0 and num_shards")
        self._sharded_len = len(iterable) // num_shards
        if len(iterable) % num_shards > 0:
            self._sharded_len += 1
        self.itr = itertools.zip_longest(
            range(self._sharded_len),
            itertools.islice(iterable, shard_id, len(iterable), num_shards),
            fillvalue=fill_value,
        )

    def __len__(self):
        return self._sharded_len

    def __iter__(self):
        return self

    def __next__(self):
        return next(self.itr)[1]
