"""Python facade of the native RCCL communication engine (``hetseq_amd/_comm``).

SURVEY §2.3 / §5.8: the reference's gradient exchange is torch DDP's C++ reducer
over NCCL (controller.py:74-89) and its stats go through c10d
(controller.py:294-296).  Here the data-parallel engine (``parallel/ddp.py``)
drives a communicator of its own (``csrc/comm/comm.cpp``): bucket all-reduces
on a greatest-priority comm stream gated by events on the producer streams,
a consumer-side join, in-stream small collectives, and a watchdog that aborts
the communicator when an operation outlives ``--collective-timeout`` (or RCCL
reports an async error) so the job fails loudly instead of hanging.

Rendezvous: rank 0 draws the RCCL unique id and publishes it through the
process group's store (the job's ``tcp://`` / ``file://`` / env rendezvous),
so no extra port or file is needed.  Engine selection (``--comm-engine``):
``native`` (default on GPUs with the nccl backend) or ``c10d`` (torch's
ProcessGroupNCCL / gloo; always used on CPU).
"""
from __future__ import annotations

import atexit
import itertools
import os
import warnings
import weakref

import torch
import torch.distributed as dist

DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float64: 2, torch.int64: 3, torch.uint8: 4, torch.int32: 5}
OPS = {"sum": 0, "min": 1, "max": 2}
_ids = itertools.count()


def module():
    """The compiled engine, or None when it is not built (CPU-only checkouts)."""
    from hetseq_amd.ops import _C

    return _C.comm()  # stamp-verified load (ops/_C.py)


def _stream(s=None):
    return (s if s is not None else torch.cuda.current_stream()).cuda_stream


class NativeComm(object):
    """One RCCL communicator over the ranks of ``group`` (all of them take part in construction)."""

    def __init__(self, group=None, timeout_s=1800.0, device=None, rendezvous=True, key=None):
        """``rendezvous=False``: only the process-local part (device, comm stream) -- nothing that
        waits for another rank; :meth:`rendezvous` then exchanges the unique id and enters
        ncclCommInitRank (create() agrees across ranks in between).  ``key``: index of the store key
        the unique id travels under (create() draws it on every rank before any check can fail, so
        the ranks' keys stay aligned whatever happens on one of them)."""
        mod = module()
        if mod is None:
            raise RuntimeError("hetseq_amd._comm is not built (python -m hetseq_amd.csrc.build)")
        self.group = group or dist.group.WORLD
        self.rank = dist.get_rank(self.group)
        self.size = dist.get_world_size(self.group)
        self.device = torch.cuda.current_device() if device is None else device
        self._key = "hetseq_comm_uid_%d" % (next(_ids) if key is None else key)
        self._mod = mod
        self._c = mod.Comm(self.size, self.rank, self.device, float(timeout_s))
        # at interpreter exit (no explicit close): abort -- frees the communicator without waiting
        # for peers, while the HIP runtime is still alive (never from static destructors)
        ref = weakref.ref(self)
        atexit.register(lambda: ref() is not None and ref()._c.close(False))
        if rendezvous:
            self.rendezvous()

    def rendezvous(self):
        """The blocking RCCL rendezvous (every rank of the group must call it): rank 0 publishes the
        unique id through the c10d store, every rank fetches it and enters ncclCommInitRank."""
        store = dist.distributed_c10d._get_default_store()
        if self.rank == 0:
            store.set(self._key, self._mod.unique_id())
        uid = store.get(self._key)  # blocks until rank 0 published it (the store's own timeout applies)
        self._c.init(uid)

    # ------------------------------------------------------------------ bucket path
    def all_reduce_async(self, t, producers=(), op="sum"):
        """In-place all-reduce of contiguous ``t`` on the comm stream, ordered after the work
        enqueued so far on every stream in ``producers`` (default: the current stream; None: only
        after earlier comm-stream work)."""
        hs = [] if producers is None else ([_stream(s) for s in producers] or [_stream()])
        self._c.all_reduce_async(t.data_ptr(), t.numel(), DTYPES[t.dtype], OPS[op], hs)

    def all_gather_async(self, out, t, producers=()):
        """``out`` = concatenation over ranks of ``t``, on the comm stream after the work enqueued
        so far on every stream in ``producers`` (default: the current stream)."""
        assert out.is_contiguous() and t.is_contiguous() and out.numel() == self.size * t.numel()
        assert out.dtype == t.dtype
        hs = [_stream(s) for s in producers] or [_stream()]
        self._c.all_gather_async(t.data_ptr(), out.data_ptr(), t.numel(), DTYPES[t.dtype], hs)
        return out

    def reduce_scatter_async(self, t, producers=(), op="sum"):
        """In-place reduce-scatter of contiguous ``t`` (numel a multiple of the rank count; emulated:
        of the emulated world): rank r's piece r holds the sum, on the comm stream after ``producers``
        (default: the current stream).  An empty ``producers`` tuple orders after the current stream;
        pass ``producers=None`` to order only after earlier comm-stream work."""
        hs = [] if producers is None else ([_stream(s) for s in producers] or [_stream()])
        self._c.reduce_scatter_async(t.data_ptr(), t.numel(), DTYPES[t.dtype], OPS[op], hs)

    def wait_events(self, events):
        """The comm stream waits for raw hipEvent_t handles the caller recorded (ordering the next
        collective after exactly that work)."""
        self._c.wait_events([int(e) for e in events])

    def all_gather_inplace_async(self, t, producers=()):
        """In-place all-gather of contiguous ``t``: every rank's piece r (of ``size`` equal pieces) to
        all ranks, on the comm stream after ``producers`` (as :meth:`reduce_scatter_async`)."""
        hs = [] if producers is None else ([_stream(s) for s in producers] or [_stream()])
        self._c.all_gather_inplace_async(t.data_ptr(), t.numel(), DTYPES[t.dtype], hs)

    def torch_stream(self):
        """The comm stream as a torch stream (work enqueued on it is ordered with the collectives)."""
        s = getattr(self, "_tstream", None)
        if s is None:
            s = torch.cuda.ExternalStream(self._c.stream, device=torch.device("cuda", self.device))
            self._tstream = s
        return s

    def set_snapshot(self, dst, src):
        """Test mode: every all_reduce_async of a slice of ``src`` copies it into the same offsets
        of ``dst`` on the comm stream instead (ordering check on one GPU); ``dst=None`` ends it."""
        if dst is None:
            self._c.set_snapshot(0, 0, 0)
        else:
            assert dst.numel() == src.numel() and dst.dtype == src.dtype
            self._c.set_snapshot(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size())

    def set_emulation(self, world, channels=32, busbw_gbs=400.0, latency_us=12.0, scratch_mb=64):
        """Predict a ``world``-rank step on this 1-rank communicator (bench.py --emulate-world):
        every bucket all-reduce / row all-gather / stats all-reduce becomes the stand-in kernel of
        csrc/kernels/comm_emul.hip -- ``channels`` workgroups (RCCL's one per channel) moving the
        bytes one rank of a ``world``-rank ring receives (an all-reduce 2(W-1)/W of the payload, an
        all-gather (W-1) payloads) through HBM and resident for ``latency_us`` + bytes / ``busbw_gbs``.
        ``world`` <= 1 restores the real collectives."""
        from hetseq_amd.ops._C import hip

        if world > 1:
            self._emul_scratch = torch.empty(int(scratch_mb) << 20, dtype=torch.uint8,
                                             device=torch.device("cuda", self.device))
            self._c.set_emulation(hip().comm_emulation_fn(), int(world), int(channels), float(busbw_gbs),
                                  float(latency_us), self._emul_scratch.data_ptr(), self._emul_scratch.numel())
        else:
            self._c.set_emulation(0, 1, 1, 1.0, 0.0, 0, 0)
            self._emul_scratch = None
        self.emulated = (int(world), int(channels), float(busbw_gbs), float(latency_us)) if world > 1 else None

    emulated = None

    def wait(self, stream=None):
        """``stream`` (default current) waits for every collective issued on the comm stream."""
        self._c.wait(_stream(stream))

    # ------------------------------------------------------------------ in-stream collectives
    def all_reduce(self, t, op="sum", stream=None):
        assert t.is_contiguous()
        self._c.all_reduce(t.data_ptr(), t.numel(), DTYPES[t.dtype], OPS[op], _stream(stream))
        return t

    def broadcast(self, t, src=0, stream=None):
        assert t.is_contiguous()
        self._c.broadcast(t.data_ptr(), t.numel(), DTYPES[t.dtype], src, _stream(stream))
        return t

    def all_gather(self, out, t, stream=None):
        """``out`` = concatenation over ranks of ``t`` (``out.numel() == size * t.numel()``)."""
        assert out.is_contiguous() and t.is_contiguous() and out.numel() == self.size * t.numel()
        self._c.all_gather(t.data_ptr(), out.data_ptr(), t.numel(), DTYPES[t.dtype], _stream(stream))
        return out

    # ------------------------------------------------------------------ health
    def watch(self, stream=None):
        """Put the work enqueued on ``stream`` (default current) so far under the watchdog -- after
        a HIP-graph replay whose collectives were captured (capture itself registers nothing)."""
        self._c.watch_stream(_stream(stream))

    def check(self):
        """Raise if the watchdog aborted the communicator (timeout or async RCCL error)."""
        self._c.check()

    @property
    def aborted(self):
        return self._c.aborted

    @property
    def stream_handle(self):
        return self._c.stream

    def inject_stall(self, n=1):
        """Fault-injection hook: the watchdog treats the next ``n`` collectives as stuck."""
        self._c.inject_stall(n)

    def outstanding(self):
        return self._c.outstanding()

    def identity(self):
        """RCCL's own view of this communicator: {rccl_count, rccl_rank, rccl_device, pci_bus_id}."""
        return dict(self._c.identity())

    def busbw(self, nbytes=64 << 20, iters=5):
        """Bus bandwidth (GB/s) of an in-stream fp32 all-reduce of ``nbytes`` over this communicator:
        2 (W - 1) / W x bytes / time (ring convention); the algorithm bandwidth when W = 1."""
        x = torch.ones(nbytes // 4, dtype=torch.float32, device=torch.device("cuda", self.device))
        for _ in range(2):
            self.all_reduce(x)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            self.all_reduce(x)
        e.record()
        e.synchronize()
        t = s.elapsed_time(e) / iters * 1e-3
        f = 2.0 * (self.size - 1) / self.size if self.size > 1 else 1.0
        return round(f * nbytes / t / 1e9, 1)

    def close(self, graceful=True):
        """Destroy the communicator (every rank at the same point), or abort it when operations
        are still outstanding / ``graceful`` is False."""
        self._c.close(graceful)


def want_native(engine, device_is_cuda, group=None):
    """Resolve ``--comm-engine`` ('auto' | 'native' | 'c10d') for a process group."""
    engine = os.environ.get("HETSEQ_COMM_ENGINE", engine or "auto")
    if engine == "c10d" or not device_is_cuda:
        return False
    backend = dist.get_backend(group or dist.group.WORLD)
    if backend != "nccl":
        if engine == "native":
            warnings.warn("--comm-engine native needs the nccl (RCCL) backend; using c10d (%s)" % backend)
        return False
    if module() is None:
        if engine == "native":
            raise RuntimeError("--comm-engine native: hetseq_amd._comm is not built")
        return False
    return True


def shard_self_test(nc, group=None):
    """Check the engine's in-place collectives that the sharded update relies on (parallel/zero.py),
    on the ranks of ``group``, before the first step: a reduce-scatter whose piece r must hold the sum
    on rank r, an all-reduce of a tail beside it, and an in-place all-gather whose every piece must
    come back from its owner.  Host check once, then every rank agrees (c10d all-reduce of a failure
    count).  Returns (ok, None) or (False, reason)."""
    W, r = nc.size, nc.rank
    dev = torch.device("cuda", nc.device)
    ps, tail = 3 * 64, 17
    why = None
    try:
        base = torch.arange(W * ps + tail, dtype=torch.float32, device=dev)
        g = base * (r + 1)
        nc.reduce_scatter_async(g[:W * ps])
        nc.all_reduce_async(g[W * ps:])
        p = torch.zeros(W * ps, dtype=torch.float32, device=dev)
        p[r * ps:(r + 1) * ps] = base[r * ps:(r + 1) * ps] - 7.0 * r
        nc.all_gather_inplace_async(p)
        nc.wait()
        tot = W * (W + 1) / 2.0
        want_g = base[r * ps:(r + 1) * ps] * tot
        want_t = base[W * ps:] * tot
        want_p = base[:W * ps] - 7.0 * torch.arange(W, device=dev, dtype=torch.float32).repeat_interleave(ps)
        nc.check()
        if not torch.equal(g[r * ps:(r + 1) * ps], want_g):
            why = "reduce-scatter: rank %d's piece does not hold the sum" % r
        elif not torch.equal(g[W * ps:], want_t):
            why = "tail all-reduce: wrong sum on rank %d" % r
        elif not torch.equal(p, want_p):
            why = "in-place all-gather: wrong pieces on rank %d" % r
    except Exception as e:  # noqa: BLE001 - any failure: the replicated update
        why = "%s: %s" % (type(e).__name__, e)
    ok = _agree(why is None, group or dist.group.WORLD, dev)
    if not ok:
        why = why or "failed on another rank"
        warnings.warn("sharded optimizer update not used: native engine self-test: %s" % why)
    return ok, (None if ok else why)


# What the last create() call decided, for logs and the benchmark record:
# {"engine": "rccl-native" | "c10d", "reason": why the native engine is not in use (or None)}
LAST_STATUS = {"engine": "c10d", "reason": "not created"}


def _agree(ok, group, device):
    """True when ``ok`` holds on EVERY rank of ``group`` (one c10d all-reduce of a failure count)."""
    flag = torch.tensor([0.0 if ok else 1.0], device=device)
    dist.all_reduce(flag, group=group)
    return float(flag.item()) == 0.0


def _fault(point, rank):
    """Fault injection for the fallback tests: ``HETSEQ_COMM_FAULT=<point>:<rank>`` with point
    ``init`` (this rank fails before the RCCL rendezvous) or ``first`` (this rank's first
    all-reduce reports a wrong result)."""
    spec = os.environ.get("HETSEQ_COMM_FAULT", "")
    for item in filter(None, spec.split(";")):
        p, _, r = item.partition(":")
        if p == point and (r == "" or int(r) == rank):
            return True
    return False


def create(engine, device_is_cuda, group=None, timeout_s=1800.0, factory=None):
    """A NativeComm when the native engine works on EVERY rank, else None (c10d path).

    Construction is a cross-rank-agreed, two-round protocol, so a local failure on one rank never
    leaves the others inside the RCCL rendezvous or with a half-working engine:

    1. every rank does everything that needs no other rank -- module built, backend, injected
       ``init`` fault, and the engine's local construction (device, greatest-priority comm stream);
       the ranks agree (c10d all-reduce) before anyone waits on another rank (the unique-id store
       exchange, ncclCommInitRank), so a failure on any rank -- rank 0 included -- strands nobody;
    2. every rank fetches rank 0's unique id through the c10d store, enters the rendezvous and
       runs one all-reduce through the communicator,
       checking the result on the host; the ranks agree again, and on any failure every rank
       aborts its communicator (never waits for peers) and falls back to c10d.

    What round 1 cannot cover is a failure INSIDE ncclCommInitRank on some ranks only (the
    library's own bootstrap, whose failures normally reach every rank): the others then wait in
    the rendezvous until RCCL's bootstrap timeout, not the collective timeout.

    The outcome and the failure reason land in :data:`LAST_STATUS`.  ``factory`` replaces the
    NativeComm constructor (tests drive the protocol over gloo with a stand-in engine).
    """
    global LAST_STATUS
    key = next(_ids)  # drawn on every rank, whatever follows: the unique-id store keys stay aligned
    engine = os.environ.get("HETSEQ_COMM_ENGINE", engine or "auto")
    backend = dist.get_backend(group or dist.group.WORLD)
    if factory is None and (engine == "c10d" or not device_is_cuda or backend != "nccl"):
        want_native(engine, device_is_cuda, group)  # (warns on an explicit native request)
        LAST_STATUS = {"engine": "c10d", "reason": "engine=%s backend=%s cuda=%s" % (engine, backend, device_is_cuda)}
        return None
    rank = dist.get_rank(group)
    size = dist.get_world_size(group)
    dev = "cuda" if backend == "nccl" else "cpu"
    reason = None
    nc = None
    try:  # round 1: everything local (no rendezvous)
        if factory is None and not want_native(engine, device_is_cuda, group):
            reason = "native engine not requested or not built"
        elif _fault("init", rank):
            reason = "injected init fault on rank %d" % rank
        else:
            nc = (factory or NativeComm)(group, timeout_s=timeout_s, rendezvous=False, key=key)
    except Exception as e:  # noqa: BLE001 - any local failure turns into the agreed fallback
        reason = "%s: %s" % (type(e).__name__, e)
    if not _agree(reason is None, group, dev):
        if nc is not None:
            try:
                nc.close(False)  # never entered the rendezvous: frees the local stream
            except Exception:  # noqa: BLE001
                pass
        LAST_STATUS = {"engine": "c10d", "reason": reason or "native engine unavailable on another rank"}
        warnings.warn("native RCCL engine not used: %s; using c10d" % LAST_STATUS["reason"])
        return None
    try:  # round 2: rendezvous + one verified collective
        nc.rendezvous()
        t = torch.ones(1, device=dev)
        nc.all_reduce(t)
        if _fault("first", rank):
            t.fill_(-1.0)
        got = float(t.item())  # one host synchronisation, at setup only
        nc.check()
        if got != float(size):
            raise RuntimeError("first all-reduce returned %g, expected %d" % (got, size))
    except Exception as e:  # noqa: BLE001 - any failure turns into the agreed fallback
        reason = "%s: %s" % (type(e).__name__, e)
    if not _agree(reason is None, group, dev):
        if nc is not None:
            try:
                nc.close(False)  # abort: frees the communicator without waiting for peers
            except Exception:  # noqa: BLE001
                pass
        LAST_STATUS = {"engine": "c10d", "reason": reason or "native engine failed on another rank"}
        warnings.warn("native RCCL engine not used: %s; using c10d" % LAST_STATUS["reason"])
        return None
    LAST_STATUS = {"engine": "rccl-native", "reason": None}
    return nc
