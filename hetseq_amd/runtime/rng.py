"""Counter-based dropout RNG state for the fused kernels.

The reference reseeds torch with ``seed + num_updates`` before every update
(controller.py:426-432) so dropout masks are reproducible on resume and
identical across ranks (Q14).  The fused kernels use Philox4x32-10 keyed by
(seed, offset): ``set_seed`` is called at the same point, and every dropout
site draws a fresh ``offset``; the (seed, offset) pair is saved for the
backward pass, which regenerates the mask bit-identically.
"""
import threading

_state = threading.local()


def set_seed(seed: int):
    _state.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    _state.offset = 0


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
