"""Loader for the in-tree native extension modules.

``native()`` -> host batcher, ``h5()`` -> HDF5 shard IO, ``hip()`` -> gfx950
kernels.  Modules are built in-tree by :mod:`hetseq_amd.csrc.build` (see
``__graft_entry__.build``); if one is missing we try to build it once.

Policy for the GPU path: when a CUDA/HIP device is present and the fused
kernels are requested, a missing or unloadable ``_hip`` module is a hard
error (``HipKernelsUnavailable``) -- there is no silent eager fallback on a
GPU box.  On CPU-only hosts the model runs its torch-op reference path.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_LOCK = threading.Lock()
_CACHE: dict = {}


class HipKernelsUnavailable(RuntimeError):
    pass


def _load(name, builder):
    with _LOCK:
        if name in _CACHE:
            return _CACHE[name]
        try:
            mod = importlib.import_module("hetseq_amd." + name)
        except ImportError:
            if os.environ.get("HETSEQ_NO_AUTOBUILD"):
                raise
            from hetseq_amd.csrc import build as _build

            getattr(_build, builder)()
            importlib.invalidate_caches()
            mod = importlib.import_module("hetseq_amd." + name)
        _CACHE[name] = mod
        return mod


def native():
    return _load("_native", "build_native")


def h5():
    return _load("_h5", "build_h5")


def hip():
    try:
        return _load("_hip", "build_hip")
    except Exception as e:  # pragma: no cover - exercised on broken installs only
        raise HipKernelsUnavailable("hetseq_amd HIP kernels (_hip) could not be loaded: %s" % e) from e


def gpu_available() -> bool:
    return torch.cuda.is_available()


def use_fused(t: torch.Tensor) -> bool:
    """Fused HIP path is used for tensors on a GPU unless disabled by env."""
    if not t.is_cuda:
        return False
    if os.environ.get("HETSEQ_DISABLE_FUSED", "0") == "1":
        return False
    hip()  # fail loudly on a GPU box without the kernels
    return True


def stream_handle() -> int:
    """Raw handle of the current HIP stream of the current device.  Every kernel launch asks
    for it, so it skips the Python Stream-object construction of torch.cuda.current_stream()
    (~10 us per call, measured with cProfile: ~1 ms of host time per BERT-base step)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


DT_F32, DT_BF16 = 0, 1


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return DT_F32
    if t.dtype == torch.bfloat16:
        return DT_BF16
    raise TypeError("HIP kernels support float32 and bfloat16 only, got %s" % t.dtype)
