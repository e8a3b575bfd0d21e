"""Flat parameter / gradient storage.

Every trainable parameter of a model is re-homed into ONE contiguous fp32
buffer (``store.param``) and its ``.grad`` into one contiguous fp32 buffer
(``store.grad``); ``p.data`` and ``p.grad`` become views.  This is the
memory layout everything else is designed around:

* the optimizer is one vectorised kernel over the whole buffer (no per-tensor
  Python loop, reference optim.py:172-229);
* the gradient-norm / clip is one reduction over one buffer;
* data-parallel buckets are contiguous slices of ``store.grad`` -- all-reduce
  runs in place, zero-copy (hetseq_amd/parallel/ddp.py);
* zero_grad is one launch -- lazily, only over the regions the next backward does not
  overwrite (see ``cover``);
* an optional bf16 ``shadow`` buffer (same offsets) holds the compute copy
  of the weights for ``--dtype bf16``; the optimizer kernel refreshes it.

Modules may declare contiguity groups (``_flat_groups``: lists of parameters
that must be adjacent, e.g. the Q/K/V projection weights) so a fused kernel
can address them as one tensor (``store.combined``).  Group starts and
standalone tensors are aligned to 64 elements (256 B).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

ALIGN = 64


def _align(n, a=ALIGN):
    return (n + a - 1) // a * a


def bisect_chunk(chunks, off):
    """Index of the (lo, hi) range of ``chunks`` holding element ``off`` (-1: none)."""
    import bisect

    i = bisect.bisect_right([lo for lo, _ in chunks], off) - 1
    return i if i >= 0 and off < chunks[i][1] else -1


CHUNK_ALIGN = 4096  # update-chunk starts (elements): whole W-piece splits for W | 64 (parallel/zero.py)


class FlatParamStore(object):
    def __init__(self, module, device=None, shadow_dtype=None):
        named = OrderedDict()
        seen = set()
        for name, p in module.named_parameters():
            if id(p) in seen or not p.requires_grad:
                continue
            seen.add(id(p))
            named[name] = p
        groups = {}
        for m in module.modules():
            for g in getattr(m, "_flat_groups", ()):
                for p in g:
                    groups[id(p)] = g
        order, placed = [], set()
        for name, p in named.items():
            if id(p) in placed:
                continue
            g = groups.get(id(p))
            members = list(g) if g is not None else [p]
            order.append(members)
            placed.update(id(q) for q in members)
        dev = torch.device(device) if device is not None else next(iter(named.values())).device
        # the model's update chunks (staged / sharded updates) start on CHUNK_ALIGN boundaries, so a
        # chunk splits into W equal aligned pieces with no remainder
        firsts = set()
        ug = getattr(module, "update_groups", None)
        gg = getattr(module, "grad_groups", None)  # finer groups the DP engine may reduce on their own
        pos = {id(q): i for i, m in enumerate(order) for q in m}
        groups_ = ((ug() or []) if callable(ug) else []) + ((gg() or []) if callable(gg) else [])
        for g in groups_:
            ps = [p for p in g if id(p) in pos]
            if ps:
                firsts.add(id(min(ps, key=lambda p: pos[id(p)])))
        offsets, cur = OrderedDict(), 0
        for members in order:
            cur = _align(cur, CHUNK_ALIGN) if any(id(q) in firsts for q in members) else _align(cur)
            for q in members:
                offsets[id(q)] = cur
                cur += q.numel()
        total = _align(cur, CHUNK_ALIGN) if firsts else _align(cur)
        self.numel = total
        self.device = dev
        self.param = torch.zeros(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.params = []
        self.names = []
        self.offsets = offsets
        name_of = {id(p): n for n, p in named.items()}
        with torch.no_grad():
            for members in order:
                for q in members:
                    off, n = offsets[id(q)], q.numel()
                    self.param[off : off + n].copy_(q.detach().reshape(-1).to(dev, torch.float32))
                    q.data = self.param[off : off + n].view(q.shape)
                    q.grad = self.grad[off : off + n].view(q.shape)
                    self.params.append(q)
                    self.names.append(name_of[id(q)])
        self.shadow = None
        if shadow_dtype is not None:
            self.shadow = torch.empty(total, dtype=shadow_dtype, device=dev)
            self.sync_shadow()

    # ------------------------------------------------------------ views
    def offset(self, p):
        return self.offsets[id(p)]

    def shadow_view(self, p):
        if self.shadow is None:
            return p.detach()
        off = self.offsets[id(p)]
        return self.shadow[off : off + p.numel()].view(p.shape)

    def combined(self, params, shape, shadow=False):
        """A single view over adjacent parameters (None if not adjacent)."""
        off = self.offsets.get(id(params[0]))
        if off is None:
            return None
        cur = off
        for p in params:
            if self.offsets.get(id(p)) != cur:
                return None
            cur += p.numel()
        buf = self.shadow if (shadow and self.shadow is not None) else self.param
        return buf[off:cur].view(shape)

    def grad_slice(self, p):
        off = self.offsets[id(p)]
        return self.grad[off : off + p.numel()]

    def grad_view(self, p):
        off = self.offsets[id(p)]
        return self.grad[off : off + p.numel()].view(p.shape)

    def combined_grad(self, params, shape):
        off = self.offsets.get(id(params[0]))
        cur = off
        for p in params:
            if self.offsets.get(id(p)) != cur:
                return None
            cur += p.numel()
        return self.grad[off:cur].view(shape)

    # Direct gradients: fused backward kernels accumulate parameter gradients
    # straight into ``self.grad`` (GEMM beta=1, kernel-side accumulate flags,
    # atomics) and return None to autograd, so no per-parameter ``grad += new``
    # pass runs.  Autograd still runs the (empty) AccumulateGrad node, whose
    # post-accumulate-grad hook is the data-parallel readiness signal.

    # ------------------------------------------------------------ ops
    # True from zero_grad() until the end of the first backward after it (end_fresh, queued by the
    # first consumer): a weight gradient that is the only writer of its region may store instead of
    # accumulating (the fused layer backward's weight-gradient products, ops/bert_ops.py) -- the
    # zeros need not be read back.
    grads_zero = False
    _fresh_end_queued = False

    # Lazy zero_grad: the regions registered with cover() are OVERWRITTEN by the first backward after
    # zero_grad (the fused layers' weight-gradient GEMMs and the tied decoder store in that backward,
    # ops/bert_ops.py), so a lazy zero_grad clears only the rest of the buffer (one launch) and leaves
    # them pending.  A writer of a pending region that accumulates instead (a second micro-batch, a
    # path without the side stream) calls ensure_zero() first; one that stores calls mark_stored();
    # whatever is still pending when the backward ends (end_fresh) or the gradients are read
    # (flush_lazy: norm, step, data-parallel buckets) is cleared then.  BERT-base: 6 MB cleared per
    # step instead of 440 MB.
    _cover: dict = None     # offset -> numel of the covered regions
    _zero_tab = None        # (table tensor, blocks) of the complement, rebuilt when _cover changes
    _pending: dict = None   # covered regions not written since the last lazy zero_grad

    def cover(self, *views):
        """Register gradient views the first backward after zero_grad overwrites (store-mode writers)."""
        if self._cover is None:
            self._cover = {}
        for v in views:
            off = (v.data_ptr() - self.grad.data_ptr()) // 4
            if off % 4 or v.numel() % 4 or not (0 <= off and off + v.numel() <= self.numel):
                continue  # (float4 granularity only)
            if self._cover.get(off) != v.numel():
                self._cover[off] = v.numel()
                self._zero_tab = None

    def _complement_table(self):
        if self._zero_tab is None:
            chunk = 4096 * 4  # floats per block
            rows, cur = [], 0
            for off, n in sorted(self._cover.items()) + [(self.numel, 0)]:
                for lo in range(cur, off, chunk):
                    rows.append((lo // 4, min(off, lo + chunk) // 4))
                cur = max(cur, off + n)
            tab = torch.tensor(rows if rows else [(0, 0)], dtype=torch.int64, device=self.device)
            self._zero_tab = (tab, len(rows))
        return self._zero_tab

    def zero_grad(self, lazy=False):
        if self.staged_pending():
            # the staged update still reads the gradients: clear them on its stream, after it, and
            # make the LAST chunk's fence cover the clearing (the forward waits for that fence before
            # the backward that writes them; params_ready waits for everything)
            from hetseq_amd.optim.optimizers import update_stream

            st = self._update_stream or update_stream(self.device)
            with torch.cuda.stream(st):
                self._zero_now(lazy)
                ev = torch.cuda.Event()
                ev.record(st)
            self._fences[-1] = ev
            return
        self._zero_now(lazy)

    def _zero_now(self, lazy):
        if (lazy and self._cover and self.grad.is_cuda and self.numel % 4 == 0
                and not torch.cuda.is_current_stream_capturing()):
            from hetseq_amd.ops._C import hip, stream_handle

            tab, nblk = self._complement_table()
            hip().zero_segs(self.grad.data_ptr(), tab.data_ptr(), nblk, stream_handle())
            self._pending = dict(self._cover)
        else:
            self.grad.zero_()
            self._pending = None
        self.grads_zero = True
        # re-attach views in case something replaced p.grad (pointer compares, every path)
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() != self.grad.data_ptr() + 4 * self.offsets[id(p)]:
                off = self.offsets[id(p)]
                p.grad = self.grad[off : off + p.numel()].view(p.shape)

    def claim_fresh(self):
        """Inside a backward: whether gradients are still all zero from zero_grad(); the first call
        queues end_fresh() for the end of this backward (later backwards accumulate)."""
        if not self.grads_zero:
            return False
        if not self._fresh_end_queued:
            self._fresh_end_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self.end_fresh)
        return True

    def end_fresh(self):
        self.grads_zero = False
        self._fresh_end_queued = False
        self.flush_lazy()

    def mark_stored(self, view):
        """A store-mode writer has been enqueued for ``view``: its region needs no zeroing."""
        if self._pending:
            self._pending.pop((view.data_ptr() - self.grad.data_ptr()) // 4, None)

    def ensure_zero(self, view):
        """About to ACCUMULATE into ``view`` (on the current stream): clear it first if a lazy zero_grad
        left it pending."""
        if self._pending:
            off = (view.data_ptr() - self.grad.data_ptr()) // 4
            n = self._pending.pop(off, None)
            if n is not None:
                self.grad[off:off + n].zero_()

    def flush_range(self, lo, hi):
        """flush_lazy for the pending regions inside [lo, hi) (a data-parallel bucket about to be reduced)."""
        if self._pending:
            for off, n in list(self._pending.items()):
                if off < hi and off + n > lo:
                    self.grad[off:off + n].zero_()
                    del self._pending[off]

    def flush_lazy(self):
        """Clear every region a lazy zero_grad left pending and no writer claimed (normally none)."""
        if self._pending:
            for off, n in list(self._pending.items()):
                self.grad[off:off + n].zero_()
            self._pending = None

    # ------------------------------------------------------------ staged update
    # The optimizer can run an update chunk by chunk on a stream of its own (optim/optimizers.py,
    # ``staged``), overlapped with the next forward: chunk i's parameters -- and what an update hook
    # derives from them on that stream (the h3p weight planes) -- may be read once the forward has
    # waited for chunk i's fence (param_ready).  Chunks are set by the model, in the order its
    # forward first reads them (BertForPreTraining: embeddings, each encoder layer, the heads).
    chunks = None   # [(lo, hi)] covering [0, numel), ascending
    _update_stream = None  # the stream the last staged update ran on (zero_grad queues behind it)
    shard = None    # parallel/zero.py ShardPlan: the elements this rank updates (sharded optimizer)
    _fences = None  # per chunk: an event recorded after its update (None: nothing pending)
    _hooks = None   # per chunk: [fn()] run on the updating stream after the chunk's update

    def set_chunks(self, groups):
        """Chunk boundaries from groups of parameters (each group contiguous in the buffer, groups
        in buffer order).  Returns False (staging unavailable) if they do not tile the buffer."""
        ranges = []
        for ps in groups:
            ps = [p for p in ps if id(p) in self.offsets]
            if not ps:
                continue
            lo = min(self.offsets[id(p)] for p in ps)
            hi = max(self.offsets[id(p)] + p.numel() for p in ps)
            ranges.append((lo, hi))
        if not ranges:
            return False
        ranges.sort()
        # extend each range to the next one's start (alignment gaps), the first to 0, the last to numel
        tiled = []
        for i, (lo, hi) in enumerate(ranges):
            nlo = 0 if i == 0 else tiled[-1][1]
            nhi = ranges[i + 1][0] if i + 1 < len(ranges) else self.numel
            if lo < nlo or hi > nhi or nlo % ALIGN or nhi % ALIGN:
                return False
            tiled.append((nlo, nhi))
        covered = sum(hi - lo for lo, hi in tiled)
        if covered != self.numel or sum(p.numel() for p in self.params) > covered:
            return False
        owners = [bisect_chunk(tiled, self.offsets[id(p)]) for p in self.params]
        if any(o < 0 for o in owners):
            return False
        self.chunks = tiled
        self._fences = [None] * len(tiled)
        self._hooks = [[] for _ in tiled]
        return True

    def chunk_of(self, p):
        return bisect_chunk(self.chunks, self.offsets[id(p)]) if self.chunks else -1

    def add_update_hook(self, chunk, fn):
        """Run ``fn()`` on the updating stream after every update of ``chunk`` (every chunk's
        hooks also run, in chunk order, after an unstaged update)."""
        self._hooks[chunk].append(fn)

    def has_hooks(self, chunk):
        return self._hooks is not None and bool(self._hooks[chunk])

    def run_hooks(self, chunk=None):
        if self._hooks is None:
            return
        for i in (range(len(self._hooks)) if chunk is None else (chunk,)):
            for fn in self._hooks[i]:
                fn()

    # Bumped by every update that changes ``param`` through raw kernels (optimizer steps, the
    # data-parallel broadcast): derived copies (h3p weight planes) are current iff made at this
    # epoch and at the tensor's version (torch ops bump that).
    epoch = 0

    def bump(self):
        self.epoch += 1

    def stamp(self):
        """The state a derived copy of the parameters is current for."""
        return (self.epoch, self.param._version)

    def staged_pending(self):
        return self._fences is not None and any(e is not None for e in self._fences)

    def param_ready(self, chunk):
        """The current stream waits for ``chunk``'s staged update (no-op when none is pending)."""
        if self._fences is not None and 0 <= chunk < len(self._fences) and self._fences[chunk] is not None:
            torch.cuda.current_stream(self.device).wait_event(self._fences[chunk])
            from hetseq_amd.runtime import streams

            other = streams.chain_stream()  # (a half-batch chain forked once, without per-layer forks)
            if other is not None:
                other.wait_event(self._fences[chunk])
            self._fences[chunk] = None

    def params_ready(self):
        """The current stream waits for every pending staged update (any reader that is not a
        chunk-aware forward: checkpoints, evaluation, unfused paths, graph capture)."""
        if self._fences is not None:
            for i in range(len(self._fences)):
                self.param_ready(i)

    def cast_shadow(self, lo, hi):
        """Refresh the bf16 shadow of elements [lo, hi) from the fp32 parameters (current stream)."""
        if self.shadow is None or hi <= lo:
            return
        if self.param.is_cuda and self.shadow.dtype == torch.bfloat16 and lo % 4 == 0 and (hi - lo) % 4 == 0:
            from hetseq_amd.ops._C import hip, stream_handle

            hip().cast_f32_bf16(self.param.data_ptr() + 4 * lo, self.shadow.data_ptr() + 2 * lo, hi - lo,
                                stream_handle())
        else:
            with torch.no_grad():
                self.shadow[lo:hi].copy_(self.param[lo:hi])

    def sync_shadow(self):
        if self.shadow is None:
            return
        with torch.no_grad():
            if self.param.is_cuda and self.shadow.dtype == torch.bfloat16:
                from hetseq_amd.ops._C import hip, stream_handle

                hip().cast_f32_bf16(self.param.data_ptr(), self.shadow.data_ptr(), self.numel, stream_handle())
            else:
                self.shadow.copy_(self.param)

    def checksum(self):
        """fp64 sum of every parameter, behind any pending staged update (its in-place all-gathers
        run on the comm stream; a checksum read beside them would see half-gathered parameters)."""
        self.params_ready()
        return self.param.double().sum()

    def segments(self):
        """[(offset, numel)] per parameter, in buffer order."""
        return [(self.offsets[id(p)], p.numel()) for p in self.params]
