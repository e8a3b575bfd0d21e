"""HIP-graph capture of the whole training update (``--hip-graph``).

One BERT update is ~400 kernel launches driven by Python; with bf16 the GPU
finishes them faster than the host can enqueue them.  The update has static
shapes, so it is captured once into a HIP graph (``torch.cuda.graph`` records
the HIP stream, including the autograd backward and the library GEMMs) and
replayed: one launch per update instead of ~400.

What may change between updates is kept in device memory the graph reads:
* the batch -> copied into static input buffers before each replay;
* the dropout seed (``args.seed + num_updates``) -> ``rng.enable_device_seed``:
  the kernels read it through ``g_seed_dev`` instead of a baked-in argument;
  the per-site Philox offsets are a fixed sequence, so they may be baked in;
* the learning rate and Adam's bias-corrected step size -> a device pair the
  fused Adam kernel reads (``_Optimizer.enable_device_hyper``).
Host values are staged through a small ring of pinned buffers
(:class:`HostToDevice`) so a refresh never overwrites a copy still in flight.
Outputs (loss statistics, grad norm) are cloned after each replay, because the
next replay overwrites them.
"""
from __future__ import annotations

import torch


class HostToDevice(object):
    """A device tensor refreshed from host values through a ring of pinned staging buffers."""

    def __init__(self, n, dtype, device, depth=4):
        self.dev = torch.zeros(n, dtype=dtype, device=device)
        self._host = [torch.zeros(n, dtype=dtype, pin_memory=True) for _ in range(depth)]
        self._events = [None] * depth
        self._slot = 0

    def push(self, values):
        k = self._slot
        self._slot = (k + 1) % len(self._host)
        ev = self._events[k]
        if ev is not None:
            ev.synchronize()  # the copy that last read this slot has finished (normally long ago)
        buf = self._host[k]
        for i, v in enumerate(values):
            buf[i] = v
        self.dev.copy_(buf, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._events[k] = ev


class GraphedStep(object):
    """Capture-once / replay-many wrapper around a step body ``fn(static_inputs) -> outputs``.

    ``outputs`` is a tuple of device tensors; ``run`` returns clones of them.
    """

    def __init__(self, fn, capture_error_mode="global"):
        self.fn = fn
        self.mode = capture_error_mode
        self.graph = None
        self.static_in = None
        self.static_out = None
        self.signature = None

    @staticmethod
    def _sig(inputs):
        return tuple((tuple(t.shape), t.dtype) for t in inputs)

    def matches(self, inputs):
        return self.graph is None or self._sig(inputs) == self.signature

    def run(self, inputs):
        if self.graph is None:
            self.static_in = [t.clone() for t in inputs]
            self.signature = self._sig(inputs)
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode=self.mode):
                with _CaptureProbe():
                    self.static_out = self.fn(self.static_in)
        else:
            for dst, src in zip(self.static_in, inputs):
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return tuple(t.clone() for t in self.static_out)


class _CaptureProbe(object):
    """HETSEQ_CAPTURE_DEBUG=1: report the first kernel-library call after which the capture stream's
    capture is no longer active (the call that invalidated it), with its Python stack."""

    def __enter__(self):
        import os

        self.on = os.environ.get("HETSEQ_CAPTURE_DEBUG") == "1"
        if not self.on:
            return self
        import traceback

        from hetseq_amd.ops._C import hip

        self.mod = hip()
        self.origin = torch.cuda.current_stream().cuda_stream
        self.saved = {}
        state = {"reported": False, "last": None}
        status = self.mod.capture_status
        origin = self.origin

        def report(what, name):
            if not state["reported"]:
                state["reported"] = True
                print("| capture probe: %s %s (previous call %s)\n%s"
                      % (what, name, state["last"], "".join(traceback.format_stack(limit=14))), flush=True)

        def wrap(name, fn):
            def probe(*a, **k):
                st = status(origin)
                if st != 1:
                    report("capture status %d before" % st, name)
                try:
                    out = fn(*a, **k)
                except Exception as e:
                    report("exception %r in" % (str(e).splitlines()[0],), name)
                    raise
                st = status(origin)
                if st != 1:
                    report("capture status %d after" % st, name)
                state["last"] = name
                return out
            return probe

        for name in dir(self.mod):
            fn = getattr(self.mod, name)
            if callable(fn) and not name.startswith("_") and name not in ("capture_status", "end_capture"):
                self.saved[name] = fn
                setattr(self.mod, name, wrap(name, fn))
        return self

    def __exit__(self, *exc):
        if self.on:
            for name, fn in self.saved.items():
                setattr(self.mod, name, fn)
        return False
