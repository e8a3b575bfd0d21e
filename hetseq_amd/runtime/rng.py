"""Counter-based dropout RNG state for the fused kernels.

The reference reseeds torch with ``seed + num_updates`` before every update
(controller.py:426-432) so dropout masks are reproducible on resume and
identical across ranks (Q14).  The fused kernels use Philox4x32-10 keyed by
(seed, offset): ``set_seed`` is called at the same point, and every dropout
site draws a fresh ``offset``; the (seed, offset) pair is saved for the
backward pass, which regenerates the mask bit-identically.
"""
import threading

import torch

_state = threading.local()


_device_seed = None  # HostToDevice when the kernels read the seed from device memory (HIP graphs)


def enable_device_seed(device):
    """Make every dropout kernel read the seed from a device word (graph replays re-seed through it)."""
    global _device_seed
    from hetseq_amd.ops._C import hip
    from hetseq_amd.runtime.graphs import HostToDevice

    if _device_seed is None:
        _device_seed = HostToDevice(1, torch.int64, device)
        hip().set_seed_ptr(_device_seed.dev.data_ptr())
    if hasattr(_state, "seed"):
        _device_seed.push([_to_i64(_state.seed)])


def disable_device_seed():
    global _device_seed
    if _device_seed is not None:
        from hetseq_amd.ops._C import hip

        hip().set_seed_ptr(0)
        _device_seed = None


def _to_i64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


def set_seed(seed: int):
    _state.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    _state.offset = 0
    if _device_seed is not None:
        _device_seed.push([_to_i64(_state.seed)])


def get_seed() -> int:
    if not hasattr(_state, "seed"):
        set_seed(0)
    return _state.seed


def next_offset(n: int = 1) -> int:
    """Reserve ``n`` consecutive Philox counter-hi values for one dropout site."""
    if not hasattr(_state, "seed"):
        set_seed(0)
    off = _state.offset
    _state.offset += int(n)
    return off


def fork():
    """(seed, offset) pair for one dropout site."""
    return get_seed(), next_offset(1 << 8)
