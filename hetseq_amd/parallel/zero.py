"""Sharded optimizer update for the flat-bucket data-parallel engine (ZeRO stage 1).

Reference: every rank of the reference runs the whole optimizer on all-reduced gradients
(controller.py:74-89 wraps the model in DDP, optim.py:162-231 steps every parameter on every
rank).  Here, with ``--shard-optimizer`` (on by default for data-parallel Adam runs):

* each gradient bucket [lo, hi) of ``parallel/ddp.py`` is split into W equal, 64-element-aligned
  pieces covering [lo, lo + W ps) -- rank r owns piece r -- plus a short tail (< 64 W elements)
  that every rank owns;
* the backward exchanges each bucket with an in-place REDUCE-SCATTER of the pieces (the native RCCL
  engine; half an all-reduce's traffic) and an all-reduce of the tail;
* the gradient norm is the sum of squares over the owned pieces (tails counted by rank 0), one
  fp64 all-reduce, then the usual clip coefficient;
* Adam updates only the owned elements (1/W of the update per rank), and the updated pieces are
  ALL-GATHERED in place -- per update chunk (embeddings, each encoder layer, the heads) on the comm
  stream, each chunk fenced (runtime/flat.py ``param_ready``), so the gather of layer i overlaps the
  next forward of layers < i;
* the sparsely exchanged embedding tables (parallel/tied.py) stay REPLICATED: their dense part (the
  tied decoder's gradient) is all-reduced, the gathered rows are added on every rank, and every rank
  runs Adam over the whole region -- the tables are the first thing the next forward reads, and
  re-gathering 94 MB there (BERT-base) would put a whole all-gather in front of it, where the update
  of 23 M elements costs ~0.1 ms.

Checkpoints stay in the unsharded ``torch.optim`` layout: ``consolidate()`` (every rank) all-gathers
the Adam moments before the master writes them.  Under ``--emulate-world W`` (one real rank) the plan
is rank 0's of W, the collectives are the stand-in kernels, and the pieces of the other W-1 ranks are
never updated: the run times a rank's work, its numerics are not a training run's.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

ALIGN = 64


class Region(object):
    __slots__ = ("lo", "hi", "ps", "body", "reduce")

    def __init__(self, lo, hi, world, reduce):
        self.lo, self.hi, self.reduce = lo, hi, reduce
        # piece size (0: the whole region is tail -- replicated, as the sparse tables are)
        self.ps = ((hi - lo) // world) // ALIGN * ALIGN if reduce else 0
        self.body = lo + world * self.ps

    def __repr__(self):
        return "Region(%d, %d, ps=%d, body=%d, reduce=%s)" % (self.lo, self.hi, self.ps, self.body, self.reduce)


class ShardPlan(object):
    """Which elements of the flat store rank ``rank`` of ``world`` updates.  ``buckets``: the
    gradient buckets' (lo, hi) ranges (reduce-scattered); ``tables``: ranges whose gradients are
    already complete on every rank (the sparse embedding exchange)."""

    def __init__(self, store, buckets, tables, world, rank, comm=None, group=None):
        self.store, self.world, self.rank = store, int(world), int(rank)
        self.comm, self.group = comm, group
        regs = [Region(lo, hi, self.world, True) for lo, hi in buckets]
        regs += [Region(lo, hi, self.world, False) for lo, hi in tables]
        self.regions = sorted(regs, key=lambda r: r.lo)
        for a, b in zip(self.regions, self.regions[1:]):
            assert a.hi <= b.lo, "overlapping shard regions"
        self.by_range = {(r.lo, r.hi): r for r in self.regions}
        self._partials = None

    # ------------------------------------------------------------------ ownership
    def piece(self, r):
        return r.lo + self.rank * r.ps, r.lo + (self.rank + 1) * r.ps

    def regions_in(self, lo, hi):
        return [r for r in self.regions if r.lo >= lo and r.hi <= hi]

    def owned(self, lo=0, hi=None):
        """Element ranges this rank updates inside [lo, hi): its piece of every region, every tail."""
        hi = self.store.numel if hi is None else hi
        out = []
        for r in self.regions_in(lo, hi):
            a, b = self.piece(r)
            if b > a:
                out.append((a, b))
            if r.hi > r.body:
                out.append((r.body, r.hi))
        return out

    def norm_segments(self):
        """Ranges whose squares this rank contributes to the gradient norm: its pieces, and the
        (replicated) tails on rank 0 only -- over the ranks, every element exactly once."""
        out = []
        for r in self.regions:
            a, b = self.piece(r)
            if b > a:
                out.append((a, b))
            if self.rank == 0 and r.hi > r.body:
                out.append((r.body, r.hi))
        return out

    # ------------------------------------------------------------------ collectives
    def reduce_bucket(self, lo, hi, producers):
        """The backward's exchange of bucket [lo, hi) on the native engine: reduce-scatter of the
        pieces, all-reduce of the tail."""
        r = self.by_range[(lo, hi)]
        g = self.store.grad
        if r.ps > 0:
            self.comm.reduce_scatter_async(g[r.lo:r.body], producers=producers)
        if r.hi > r.body:
            self.comm.all_reduce_async(g[r.body:r.hi], producers=producers)

    def gather(self, buf, regions):
        """All-gather the pieces of ``regions`` of ``buf`` (param or a moment buffer) in place: on the
        comm stream after its earlier work (native engine), else on the current stream (c10d)."""
        for r in regions:
            if r.ps == 0:
                continue
            if self.comm is not None and buf.is_cuda:
                self.comm.all_gather_inplace_async(buf[r.lo:r.body], producers=None)
            else:
                views = [buf[r.lo + k * r.ps:r.lo + (k + 1) * r.ps] for k in range(self.world)]
                mine = views[self.rank].clone()
                dist.all_gather(views, mine, group=self.group)

    def all_reduce_scalar(self, t):
        if self.comm is not None and t.is_cuda:
            self.comm.all_reduce(t)
        else:
            dist.all_reduce(t, group=self.group)

    # ------------------------------------------------------------------ norm
    def grad_norm(self, scale, max_norm, out):
        """out[0:3] = (norm of scale * g, combined multiplier, clip coefficient), as the unsharded
        ``clip_grad_norm`` -- the squares summed over the shards in a different order (rounding)."""
        g = self.store.grad
        segs = self.norm_segments()
        if g.is_cuda:
            from hetseq_amd.ops._C import hip, stream_handle

            if self._partials is None:  # (the plan is static: one segment table for the job)
                cap = hip().sumsq_blocks()
                rows, nb = [], 0
                for a, b in segs:
                    rows += [a, b, nb]
                    nb += max(1, min(cap, (b - a) // 16384))
                self._segs = torch.tensor(rows, dtype=torch.int64).to(g.device)
                self._nblk = nb
                self._partials = torch.zeros(nb + 1, dtype=torch.float64, device=g.device)
            p = self._partials
            st = stream_handle()
            hip().sumsq_segs(g.data_ptr(), self._segs.data_ptr(), len(segs), self._nblk, p.data_ptr(), st)
            tot = p[self._nblk:self._nblk + 1]
            hip().sum_partials(p.data_ptr(), self._nblk, tot.data_ptr(), st)
            self.all_reduce_scalar(tot)
            hip().norm_finalize(tot.data_ptr(), 1, scale.data_ptr(), float(max_norm), out.data_ptr(), st)
            return
        tot = torch.zeros(1, dtype=torch.float64)
        for a, b in segs:
            tot += g[a:b].double().pow(2).sum()
        self.all_reduce_scalar(tot)
        norm = scale[0].abs() * tot.sqrt().float()[0]
        clip = torch.ones((), dtype=torch.float32)
        if max_norm > 0:
            clip = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        out[0] = norm
        out[1] = scale[0] * clip
        out[2] = clip

    # ------------------------------------------------------------------ update
    def step(self, opt, gmul, staged):
        """The sharded update: per chunk, Adam on the owned elements, the in-place all-gather of the
        chunk's pieces (and the bf16 shadow's re-cast), the chunk's update hooks, its fence.  The
        replicated regions (the sparse tables) are updated on the current stream -- the next forward
        reads them first, and the comm stream meanwhile starts the chunks' gathers."""
        s = self.store
        chunks = s.chunks if s.chunks is not None else [(0, s.numel)]
        if getattr(self, "_per_chunk", None) is None or len(self._per_chunk) != len(chunks):
            rep = [r for r in self.regions if r.ps == 0 and not r.reduce]
            self._replicated = [(r.lo, r.hi) for r in rep]
            self._per_chunk = [([(a, b) for a, b in self.owned(lo, hi) if (a, b) not in self._replicated],
                                self.regions_in(lo, hi)) for lo, hi in chunks]
        native = self.comm is not None and s.param.is_cuda
        if native:
            st = self.comm.torch_stream()
            cur = torch.cuda.current_stream(s.device)
            ready = torch.cuda.Event()
            ready.record(cur)  # the reduced gradients and the norm
        for a, b in self._replicated:
            opt._step_range(gmul, a, b)
            s.cast_shadow(a, b)
        if native:
            rep_done = torch.cuda.Event()
            rep_done.record(cur)
            st.wait_event(ready)
            ctx = torch.cuda.stream(st)
        else:
            st, ctx = None, _nullctx()
        with ctx:
            for i, (owned, regs) in enumerate(self._per_chunk):
                for a, b in owned:
                    opt._step_range(gmul, a, b)
                self.gather(s.param, regs)
                if s.shadow is not None:
                    for r in regs:
                        if (r.lo, r.hi) not in self._replicated:
                            s.cast_shadow(r.lo, r.hi)
                if native and s.chunks is not None and s.has_hooks(i) and any(
                        r.ps == 0 and not r.reduce for r in regs):
                    st.wait_event(rep_done)  # (hooks reading a replicated region)
                s.run_hooks(i) if s.chunks is not None else s.run_hooks()
                if native and staged and s.chunks is not None:
                    ev = torch.cuda.Event()
                    ev.record(st)
                    s._fences[i] = ev
            if native:
                # later comm-stream work (the deferred zero_grad, the next step's exchanges) follows
                # the replicated regions' update, which reads their gradients
                st.wait_event(rep_done)
        if native:
            s._update_stream = st
            if not (staged and s.chunks is not None):
                torch.cuda.current_stream(s.device).wait_stream(st)

    def consolidate(self, opt):
        """Every rank: all-gather the Adam moments' pieces so the master's state_dict() holds the
        whole (unsharded) optimizer state; the caller's stream waits for it."""
        for key in opt.STATE_KEYS:
            self.gather(opt._state[key], self.regions)
        if self.comm is not None and self.store.param.is_cuda:
            self.comm.wait()


class _nullctx(object):
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
