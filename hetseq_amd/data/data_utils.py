"""Data utilities (reference: data/data_utils.py:14-61).

``numpy_seed`` is the same seed-and-restore context manager.
``batch_by_size`` calls the native C++ batcher (hetseq_amd/csrc/native/
batcher.cpp) with a vector of token counts instead of a per-index Python
callback; the batch lists are identical to the reference's.
"""
from __future__ import annotations

import contextlib
import sys

import numpy as np


@contextlib.contextmanager
def numpy_seed(seed, *addl_seeds):
    """Seed the NumPy PRNG and restore its state afterwards."""
    if seed is None:
        yield
        return
    if len(addl_seeds) > 0:
        seed = int(hash((seed, *addl_seeds)) % 1e6)
    state = np.random.get_state()
    np.random.seed(seed)
    try:
        yield
    finally:
        np.random.set_state(state)


def _num_tokens_vector(indices, num_tokens_fn):
    """Token counts as an int64 vector, or a Python int when constant."""
    if isinstance(num_tokens_fn, (int, np.integer)):
        return int(num_tokens_fn)
    owner = getattr(num_tokens_fn, "__self__", None)
    const = getattr(owner, "constant_num_tokens", None) if owner is not None else None
    if const is not None:
        return int(const)
    vec = getattr(owner, "num_tokens_vector", None) if owner is not None else None
    if vec is not None:
        return np.ascontiguousarray(vec(indices), dtype=np.int64)
    return np.fromiter((int(num_tokens_fn(int(i))) for i in indices), dtype=np.int64, count=len(indices))


def batch_by_size(indices, num_tokens_fn, max_tokens=None, max_sentences=None, required_batch_size_multiple=1):
    """Mini-batches of indices bucketed by size (reference cut rule, native loop)."""
    from hetseq_amd.ops._C import native

    indices = np.ascontiguousarray(np.asarray(indices, dtype=np.int64))
    max_tokens = max_tokens if max_tokens is not None else sys.maxsize
    max_sentences = max_sentences if max_sentences is not None else sys.maxsize
    lens = _num_tokens_vector(indices, num_tokens_fn)
    try:
        return native().batch_by_size(indices, lens, int(max_tokens), int(max_sentences),
                                      int(required_batch_size_multiple))
    except RuntimeError as e:  # sample longer than max_tokens -> same error type as the reference's assert
        raise AssertionError(str(e)) from None


def batch_by_size_py(indices, num_tokens_fn, max_tokens=None, max_sentences=None, required_batch_size_multiple=1):
    """Pure-Python oracle of the reference algorithm (used by tests)."""
    max_tokens = max_tokens if max_tokens is not None else sys.maxsize
    max_sentences = max_sentences if max_sentences is not None else sys.maxsize
    bsz_mult = required_batch_size_multiple
    sample_len = 0
    sample_lens, batch, batches = [], [], []
    for idx in indices:
        n = num_tokens_fn(idx)
        sample_lens.append(n)
        sample_len = max(sample_len, n)
        assert sample_len <= max_tokens
        num_tokens = (len(batch) + 1) * sample_len
        full = len(batch) > 0 and (len(batch) == max_sentences or num_tokens > max_tokens)
        if full:
            mod_len = max(bsz_mult * (len(batch) // bsz_mult), len(batch) % bsz_mult)
            batches.append(batch[:mod_len])
            batch = batch[mod_len:]
            sample_lens = sample_lens[mod_len:]
            sample_len = max(sample_lens) if len(sample_lens) > 0 else 0
        batch.append(int(idx))
    if len(batch) > 0:
        batches.append(batch)
    return batches
