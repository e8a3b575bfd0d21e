"""Loader for the in-tree native extension modules.

``native()`` -> host batcher, ``h5()`` -> HDF5 shard IO, ``hip()`` -> gfx950
kernels.  Modules are built in-tree by :mod:`hetseq_amd.csrc.build` (see
``__graft_entry__.build``); if one is missing we try to build it once.

Policy for the GPU path: when a CUDA/HIP device is present and the fused
kernels are requested, a missing or unloadable ``_hip`` module is a hard
error (``HipKernelsUnavailable``) -- there is no silent eager fallback on a
GPU box.  On CPU-only hosts the model runs its torch-op reference path.

Integrity: before a module is imported its embedded source stamp
(``csrc/build.py``) is compared with the hash of the sources next to it.  A
stale module is rebuilt first, or -- with ``HETSEQ_NO_AUTOBUILD=1`` -- refused
with an error that names both hashes; a ``.so`` that does not belong to the
tree is never loaded.
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


class StaleModule(ImportError):
    pass


def verify_stamp(name, builder=None, so_path=None):
    """Make sure ``hetseq_amd/<name>.so`` was built from the sources in this tree: rebuild it
    (``builder``) when its stamp differs, or raise :class:`StaleModule` when rebuilding is off
    (``HETSEQ_NO_AUTOBUILD=1``) or does not help.  No-op when the sources are not present."""
    from hetseq_amd.csrc import build as _build

    try:
        have, want = _build.stamp_status(name, so_path)
    except (OSError, RuntimeError, KeyError):
        return  # sources / toolchain headers not in this checkout: nothing to compare against
    if have == want:
        return
    what = "hetseq_amd.%s: embedded source stamp %s does not match the tree (%s)" % (name, have, want)
    if builder is None or os.environ.get("HETSEQ_NO_AUTOBUILD"):
        raise StaleModule(what + "; rebuild with python -m hetseq_amd.csrc.build")
    getattr(_build, builder)()
    have = _build.embedded_hash(so_path) if so_path else _build.stamp_status(name)[0]
    if have != want:
        raise StaleModule(what + " even after a rebuild")


def _load(name, builder):
    with _LOCK:
        if name in _CACHE:
            return _CACHE[name]
        verify_stamp(name, builder)
        importlib.invalidate_caches()
        mod = importlib.import_module("hetseq_amd." + name)
        _CACHE[name] = mod
        return mod


def native():
    return _load("_native", "build_native")


def h5():
    return _load("_h5", "build_h5")


def comm():
    """The RCCL engine module, or None when it cannot be built / loaded here."""
    try:
        return _load("_comm", "build_comm")
    except (ImportError, RuntimeError):
        return None


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
