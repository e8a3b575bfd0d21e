"""Tracing / profiling helpers.

* ``range_push`` / ``range_pop``: roctx ranges (libroctx64 via ctypes) around
  embeddings, every encoder layer, the MLM decoder, the optimizer and each
  gradient bucket, visible in ``rocprofv3 --marker-trace``.  No-ops unless
  profiling is enabled (``--profile`` or ``HETSEQ_PROFILE=1``), so the hot
  loop pays nothing by default.  (The reference has a single NVTX range
  around the decoder GEMM, bert_modeling.py:546-548.)
* ``PhaseTimer``: hipEvent-based device timing per named phase, reported as
  meters (``--profile``).
"""
from __future__ import annotations

import ctypes
import os
from collections import defaultdict

import torch

_enabled = os.environ.get("HETSEQ_PROFILE", "0") == "1"
_lib = None


def enable(flag=True):
    global _enabled
    _enabled = bool(flag)


def enabled():
    return _enabled


def _roctx():
    global _lib
    if _lib is None:
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                _lib = ctypes.CDLL(name)
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        if _lib is None:
            _lib = False
    return _lib


def range_push(name):
    if not _enabled:
        return
    lib = _roctx()
    if lib:
        lib.roctxRangePushA(name.encode())


def range_pop():
    if not _enabled:
        return
    lib = _roctx()
    if lib:
        lib.roctxRangePop()


class PhaseTimer(object):
    """Accumulates device time per phase with hipEvents (resolved lazily)."""

    def __init__(self):
        self.pending = []
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    def start(self, name):
        if not (_enabled and torch.cuda.is_available()):
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return (name, ev)

    def stop(self, tok):
        if tok is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.pending.append((tok[0], tok[1], ev))

    def resolve(self):
        for name, a, b in self.pending:
            b.synchronize()
            self.totals[name] += a.elapsed_time(b)
            self.counts[name] += 1
        self.pending = []
        return {k: self.totals[k] / max(1, self.counts[k]) for k in self.totals}
