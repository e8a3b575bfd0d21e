"""Weight-gradient side stream: overlap the wgrad GEMMs with the data-gradient chain.

In a layer's backward only the data gradient (dgrad) is on the critical path:
layer i-1 needs dX of layer i, nothing needs dW until the all-reduce / optimizer.
The BERT GEMMs are small for a 256-CU chip (M = 4096 tokens -> 192..768 tiles of
128x128), so a single stream leaves CUs idle in every GEMM tail.  The fused
layer backward therefore enqueues its four weight-gradient GEMMs on a second
HIP stream (forked from the compute stream with an event wait) and lets the next
dgrad run concurrently; blocks of both fill the machine.

Ordering rules kept here:
* ``fork(device, *tensors)`` -- the side stream waits for everything enqueued on
  the compute stream so far (one event record + wait in C++, a few microseconds),
  and the inputs are kept referenced until the join, so the caching allocator
  cannot hand their memory to new compute-stream work while the side stream still
  reads it (cheaper than ``record_stream`` and no allocator-side event polling);
* ``join()`` -- the compute stream waits for the side stream and the kept inputs
  are released.  It is queued as an autograd-engine callback the first time a
  backward forks, so any consumer of the gradients after ``backward()``
  (grad-norm, optimizer, tests) is ordered;
* the data-parallel engine orders a bucket's all-reduce after both producers
  without stalling the compute stream: the native RCCL engine's comm stream
  waits on events of both streams; the c10d path issues the collective from
  the side stream after it waits for the compute stream (parallel/ddp.py).

Only gradients that go straight into the flat store use the side stream.  Under
HIP-graph capture (--hip-graph) the fork/join events are captured as graph edges
(the side stream joins the capture at the fork and leaves it at the join).
``HETSEQ_WGRAD_STREAM=0`` disables it.  The switch costs ~5 us of host time per
GEMM (raw stream get/set, one C++ event call), so host-bound configurations (bf16
without graphs) may prefer it off; ``Controller`` decides (see ``auto_enable``).
"""
from __future__ import annotations

import os

import torch

_ENABLED = os.environ.get("HETSEQ_WGRAD_STREAM", "1") == "1"
# split-K of the side-stream wgrad GEMMs.  The per-call-site choice is measured with the GEMM
# alone on the chip (4 slices for most weight gradients); running beside the dgrad chain, 2 slices
# measured best (BERT-base fp32: 16.6 ms/step vs 17.6 with the isolated choice, 19.2 with 1).
# (None = the isolated measurement; re-measured in round 5: 1 or 2 slices everywhere were slower.)
SIDE_KSPLIT = 2
# ... except the small ones (output <= 768 x 768, the attention-output projection: 36 tiles, 72
# blocks at 2 slices), which take 4: 15.431 / 15.442 / 15.451 ms/step vs 15.491 / 15.540 / 15.511
# with 2 and 15.46-15.50 with 8 (interleaved, profiles/r2_gemm_experiments.md)
SIDE_KSPLIT_SMALL = 4


def side_ksplit(M, N):
    """K split of an M x N weight-gradient GEMM on the side stream (None: the isolated measurement)."""
    if SIDE_KSPLIT is None:
        return None
    return SIDE_KSPLIT_SMALL if M * N <= 768 * 768 else SIDE_KSPLIT
# split-K of the compute-stream data-gradient GEMMs while the side stream runs the weight
# gradients beside them: the two streams fill the chip together, so the K split the isolated
# measurement picks (4 slices for the N = 768 products) only adds slab traffic and a reduction
# pass.  1 measured best (BERT-base fp32, interleaved runs: 15.53 / 15.55 ms/step vs 15.72 with the
# isolated choice, profiles/r2_gemm_experiments.md); "auto" = use the isolated measurement.
DGRAD_KSPLIT = 1
_STREAMS: dict = {}
_state = {"queued": False, "coalesce": 0}
# share one fork event between consecutive side-stream launches (bench --ab fork_co / fork_each)
COALESCE = True


def set_enabled(flag: bool):
    global _ENABLED
    _ENABLED = bool(flag)


def enabled() -> bool:
    return _ENABLED and torch.cuda.is_available()


def is_side(stream_handle: int) -> bool:
    """Whether a raw stream handle is one of the side streams (split-K workspaces are per role)."""
    return any(s.cuda_stream == stream_handle for s in _STREAMS.values())


def _new_stream(idx):
    """A process-lifetime non-blocking HIP stream of device ``idx`` (not from torch's pool)."""
    from hetseq_amd.ops._C import hip

    prev = torch.cuda.current_device()
    torch.cuda.set_device(idx)
    try:
        return torch.cuda.ExternalStream(hip().stream_create(0), device=torch.device("cuda", idx))
    finally:
        torch.cuda.set_device(prev)


def side(device) -> "torch.cuda.Stream":
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _STREAMS.get(idx)
    if s is None:
        s = _new_stream(idx)
        _STREAMS[idx] = s
    return s


def fwd2(device) -> "torch.cuda.Stream":
    """The second forward stream of ``device``: the other half-batch chain of the encoder forward
    (ops/bert_ops.py ``_layer_forward_split``).  It IS the weight-gradient side stream: that one has
    no work during the forward (the previous backward joined it), and a fifth stream would share a
    hardware queue with a busy one (GPU_MAX_HW_QUEUES = 4: compute, side, comm, copy)."""
    return side(device)


def role(stream_handle: int) -> str:
    """'side' or 'main': which engine stream a raw handle is (per-role scratch: split-K slabs)."""
    return "side" if is_side(stream_handle) else "main"


# An ordering point between two streams costs the recording stream ~6.5 us of GPU time between two
# dependent kernels (a round trip compute -> side -> compute ~27 us, tools/probes/fork_gap.py), so
# consecutive forks share one event (:class:`coalesced`).  In the training step the other stream
# fills most of that bubble (profiles/r3_forks.md).


# Half-batch chains that run through several layers without meeting (:class:`fwd_chain`): each
# half only reads its own rows, so the two streams need to meet once before the first layer and
# once after the last, not at every layer boundary (where the faster half idles until the slower
# one's LayerNorm ends, and each meeting costs an event round trip).
FWD_CHAIN = True
# Inside a chain, every later layer still orders fwd2 after the current stream's work so far (one
# event, one way: the current stream never waits): that layer's whole-batch outputs come from the
# current stream's allocator pool, which may hand out a block whose previous use -- a current-stream
# kernel enqueued after the first fork -- is still pending; fwd2 must not write its half into it
# before that kernel ran.
FWD_CHAIN_FORK = True
_chain = {"depth": 0, "forked": None, "keep": []}


class fwd_chain(object):
    """``with fwd_chain(dev): <layers>`` -- the :class:`fwd_halves` blocks inside fork the second
    half-batch chain once and do not join it; on exit (or at :func:`chain_join`) the current stream
    waits for it.  Only for layers whose whole-batch tensors outlive the block (saved for the
    backward): the second chain may still read them after a layer returns."""

    def __init__(self, device, on=True):
        self.device = device
        self.on = on and FWD_CHAIN

    def __enter__(self):
        if self.on:
            _chain["depth"] += 1
        return self

    def __exit__(self, *exc):
        if self.on:
            _chain["depth"] -= 1
            if _chain["depth"] == 0:
                chain_join(self.device)
        return False


def chain_join(device):
    """The current stream waits for an open half-batch chain (no-op when none is forked); the tensors
    the chain kept alive (:func:`chain_keep`) are released after the wait."""
    st = _chain["forked"]
    if st is not None:
        from hetseq_amd.ops._C import hip, stream_handle

        _chain["forked"] = None
        hip().stream_wait(stream_handle(), st.cuda_stream)
    _chain["keep"].clear()


def chain_fork(device):
    """Open the second half-batch chain on fwd2 unless already open (the native layer program's
    forward: its arena is the layer's own, so one fork per chain suffices -- no per-layer fork
    against allocator reuse, FWD_CHAIN_FORK)."""
    st = fwd2(device)
    if _chain["forked"] is not st:
        from hetseq_amd.ops._C import hip, stream_handle

        hip().stream_wait(st.cuda_stream, stream_handle())
        _chain["forked"] = st
    return st


def chain_stream():
    """The forked second half-batch chain's stream (None outside an open chain)."""
    return _chain["forked"]


def chain_keep(*tensors):
    """Keep tensors the second chain reads alive until it is joined (no-op outside a chain)."""
    if _chain["forked"] is not None:
        _chain["keep"].extend(t for t in tensors if t is not None)


class fwd_halves(object):
    """``with fwd_halves(dev) as halves: for h in halves: ...`` -- iteration 0 on the current stream,
    iteration 1 on :func:`fwd2` (forked from the current stream with an event wait); on exit the
    current stream waits for fwd2 -- unless inside a :class:`fwd_chain`, which forks once and joins
    at its end.  Tensors the second half allocates come from fwd2's pool."""

    def __init__(self, device):
        self.device = device
        self.gen = None

    def __enter__(self):
        from hetseq_amd.ops._C import hip, stream_handle

        self.st = fwd2(self.device)
        self.chained = _chain["depth"] > 0
        if not (self.chained and _chain["forked"] is self.st) or FWD_CHAIN_FORK:
            hip().stream_wait(self.st.cuda_stream, stream_handle())
            if self.chained:
                _chain["forked"] = self.st
        self.gen = self._halves()
        return self.gen

    def _halves(self):
        yield 0
        st = self.st
        prev = torch._C._cuda_getCurrentStream(st.device_index)
        torch._C._cuda_setStream(stream_id=st.stream_id, device_index=st.device_index, device_type=st.device_type)
        try:
            yield 1
        finally:
            torch._C._cuda_setStream(stream_id=prev[0], device_index=prev[1], device_type=prev[2])

    def __exit__(self, *exc):
        from hetseq_amd.ops._C import hip, stream_handle

        self.gen.close()  # restores the current stream if the loop left early
        if not self.chained or exc[0] is not None:
            _chain["forked"] = None
            hip().stream_wait(stream_handle(), self.st.cuda_stream)
            _chain["keep"].clear()
        return False


def reserve(device):
    """Create the weight-gradient and copy streams of ``device`` now -- before RCCL (torch's process
    group, the native engine) and torch's stream pool create theirs.  HIP hands the first
    GPU_MAX_HW_QUEUES streams of a process a hardware queue each and makes later ones share the
    least-used queue: created after RCCL's ten internal streams, the side stream landed on the
    compute stream's queue and the two serialised (BERT-base DP step 19.3 ms vs 15.1,
    profiles/r3_stream_queues.md).  The comm stream (greatest priority) gets a priority queue."""
    if device is None or device.type != "cuda" or not torch.cuda.is_available():
        return
    side(device)
    copy_stream(device)


_COPY: dict = {}


def copy_stream(device) -> "torch.cuda.Stream":
    """The process's host-to-device copy stream of ``device`` (the data loader's batch uploads).
    One per device for the whole job: a stream per epoch iterator would draw new pool streams
    and, past GPU_MAX_HW_QUEUES, land on a hardware queue shared with the compute / side / comm
    streams (profiles/r3_stream_queues.md)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _COPY.get(idx)
    if s is None:
        s = _new_stream(idx)
        _COPY[idx] = s
    return s


def engine_streams(device) -> dict:
    """Raw handles of the streams this process runs work on, by role (created ones only)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    out = {"compute": torch.cuda.current_stream(torch.device("cuda", idx)).cuda_stream}
    if idx in _STREAMS:
        out["wgrad"] = _STREAMS[idx].cuda_stream
    if idx in _COPY:
        out["copy"] = _COPY[idx].cuda_stream
    return out


def active(device) -> "torch.cuda.Stream | None":
    """The side stream if one has been forked in the current backward, else None."""
    return _STREAMS.get(device.index) if _state["queued"] else None


_KEEP: list = []


class coalesced(object):
    """``with coalesced(): ...`` -- forks inside it after the first reuse its event: the caller
    guarantees that nothing is enqueued on the current stream between them (e.g. an LN backward's
    parameter-gradient finalisation and the weight gradient that follows it)."""

    def __enter__(self):
        self.prev = _state.get("coalesce", 0)
        _state["coalesce"] = 1
        return self

    def __exit__(self, *exc):
        _state["coalesce"] = self.prev
        return False


def fork(device, *tensors) -> "torch.cuda.Stream":
    from hetseq_amd.ops._C import hip, stream_handle

    s = side(device)
    c = _state.get("coalesce", 0)
    if c != 2 or not COALESCE:
        hip().stream_wait(s.cuda_stream, stream_handle())
        if c == 1:
            _state["coalesce"] = 2
    _KEEP.extend(tensors)
    if not _state["queued"]:
        _state["queued"] = True
        torch.autograd.Variable._execution_engine.queue_callback(join)
    return s


def backward_forks(device, *tensors):
    """The bookkeeping of :func:`fork` for a caller that enqueues its own side-stream forks (the
    native layer program): the end-of-backward join is queued and ``tensors`` (read on the side
    stream) stay alive until it.  Returns the side stream."""
    s = side(device)
    _KEEP.extend(tensors)
    if not _state["queued"]:
        _state["queued"] = True
        torch.autograd.Variable._execution_engine.queue_callback(join)
    return s


def run(device, fn, *tensors):
    """fn() with the side stream current (forked from the current stream; inputs kept alive).
    Raw get/set of the current stream: the torch.cuda.stream() context costs ~20 us of host time."""
    st = fork(device, *tensors)
    prev = torch._C._cuda_getCurrentStream(st.device_index)
    torch._C._cuda_setStream(stream_id=st.stream_id, device_index=st.device_index, device_type=st.device_type)
    try:
        return fn()
    finally:
        torch._C._cuda_setStream(stream_id=prev[0], device_index=prev[1], device_type=prev[2])


def wait(device):
    """Current stream waits for the side stream (mid-backward ordering point, e.g. before the
    embedding backward accumulates into the word-embedding gradient the tied decoder's
    side-stream GEMM also writes).  Keeps the backward's join pending."""
    s = _STREAMS.get(device.index)
    if s is not None and _state["queued"]:
        from hetseq_amd.ops._C import hip, stream_handle

        hip().stream_wait(stream_handle(), s.cuda_stream)


_MARKS: dict = {}  # (device index, key) -> event recorded on the side stream in this backward


def mark(device, key):
    """Record an event on the side stream now (e.g. right after the tied decoder's weight GEMM was
    enqueued), so a later consumer waits for exactly that work (:func:`wait_mark`) instead of for
    everything the side stream holds by then."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _STREAMS.get(idx)
    if s is None or not _state["queued"]:
        return
    ev = _MARKS.get((idx, key))
    if ev is None:
        ev = torch.cuda.Event()
    ev.record(s)
    _MARKS[(idx, key)] = ev
    _MARKED.add((idx, key))


_MARKED: set = set()


def wait_mark(device, key):
    """Current stream waits for the event :func:`mark` recorded under ``key`` in this backward (or,
    without one, for the whole side stream, as :func:`wait`)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if (idx, key) in _MARKED:
        torch.cuda.current_stream(torch.device("cuda", idx)).wait_event(_MARKS[(idx, key)])
        return
    wait(device)


def join():
    """Make the current stream wait for every side stream (end of backward); release kept inputs."""
    if not _state["queued"] and not _KEEP:
        return
    from hetseq_amd.ops._C import hip

    _state["queued"] = False
    _MARKED.clear()
    for idx, s in _STREAMS.items():
        hip().stream_wait(torch._C._cuda_getCurrentRawStream(idx), s.cuda_stream)
    _KEEP.clear()
