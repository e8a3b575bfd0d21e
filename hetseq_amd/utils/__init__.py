"""Small utilities (reference: utils.py:12-37, 86-91, 167-171).

``apply_to_sample`` / ``move_to_cuda`` recurse over lists/tuples/dicts;
``move_to_cuda`` copies with ``non_blocking=True`` (pinned sources overlap
with compute) instead of the reference's blocking pageable copies.
"""
import math

import torch


def apply_to_sample(f, sample):
    if sample is None or (hasattr(sample, "__len__") and len(sample) == 0):
        return {}

    def _apply(x):
        if torch.is_tensor(x):
            return f(x)
        if isinstance(x, dict):
            return {k: _apply(v) for k, v in x.items()}
        if isinstance(x, list):
            return [_apply(v) for v in x]
        if isinstance(x, tuple):
            return tuple(_apply(v) for v in x)
        return x

    return _apply(sample)


def move_to_cuda(sample, device=None):
    def _move(t):
        if t.is_cuda and (device is None or t.device == torch.device(device)):
            return t
        return t.to(device if device is not None else "cuda", non_blocking=True)

    return apply_to_sample(_move, sample)


def item(tensor):
    if hasattr(tensor, "item"):
        return tensor.item()
    if hasattr(tensor, "__getitem__"):
        return tensor[0]
    return tensor


def get_perplexity(loss):
    try:
        return float("{:.2f}".format(math.pow(2, loss)))
    except OverflowError:
        return float("inf")
