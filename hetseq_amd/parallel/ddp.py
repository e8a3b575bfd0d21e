"""Flat-bucket data-parallel engine.

Replaces ``torch.nn.parallel.DistributedDataParallel`` (reference:
controller.py:74-89) with an engine built on the flat gradient buffer
(hetseq_amd/runtime/flat.py):

* buckets are CONTIGUOUS slices of ``store.grad`` formed in reverse
  parameter order (the order gradients become ready in backward) up to
  ``--bucket-cap-mb`` -- the all-reduce runs in place on the slice, no
  gather/scatter copies;
* each parameter's post-accumulate-grad hook counts down its bucket; ready
  buckets are launched strictly in bucket order (same collective order on
  every rank) as async ``all_reduce`` on the process group -- RCCL runs them on
  its own stream, overlapping with the rest of backward; a callback queued on
  the autograd engine waits for them at the end of backward (stream-level
  wait, no host sync on GPU);
* gradients are SUMMED, not averaged: the controller's grad-scale factor
  (reference: W / sample_size after DDP's 1/W) is folded into the fused
  optimizer as 1 / sample_size, saving a full pass over the gradients;
* ``no_sync()`` skips communication for the first update_freq-1 micro
  batches (reference: controller.py:245-258);
* the constructor broadcasts rank 0's parameters (one collective on the flat
  buffer, X3);
* on GPUs with the nccl backend the collectives go through the native RCCL
  engine (``parallel/comm.py`` over ``csrc/comm/comm.cpp``): a bucket's
  all-reduce is enqueued on a greatest-priority comm stream behind events on
  BOTH producer streams (compute and weight-gradient), the end of backward
  makes the compute stream wait for the comm stream, and a watchdog turns a
  stuck collective into an error.  ``--comm-engine c10d`` (and every CPU/gloo
  run) uses ``torch.distributed`` instead.

Bucket sizing for MI355X: with 7 xGMI links per GPU a ring all-reduce is
per-link bound; the default 25 MB (reference default) yields one bucket per
BERT layer (7.1 M params = 28 MB) so communication of layer i overlaps the
backward of layer i-1.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist

from hetseq_amd.parallel import comm as native_comm
from hetseq_amd.parallel.tied import SparseTableSync
from hetseq_amd.runtime import profiling, streams


class FlatDDP(torch.nn.Module):
    def __init__(self, module, store, process_group=None, bucket_cap_mb=25, find_unused_parameters=False,
                 broadcast=True, comm_engine="auto", timeout_s=1800.0, sparse_embedding=None, sparse_capacity=None,
                 plan_world=None, shard_optimizer=False):
        super().__init__()
        self.module = module
        self.store = store
        self.process_group = process_group or dist.group.WORLD
        self.world_size = dist.get_world_size(self.process_group)
        # world size the layout decisions (sparse tables) and the byte accounting are made for: the
        # real one, or the W a 1-rank run emulates (bench.py --emulate-world)
        self.plan_world = int(plan_world) if plan_world else self.world_size
        # native RCCL engine (None: torch.distributed); chosen identically on every rank
        # (a 1-rank group gets one only on an explicit "native" request: the single-GPU tests)
        self.comm = native_comm.create(comm_engine, store.grad.is_cuda, self.process_group, timeout_s) \
            if self.world_size > 1 or comm_engine == "native" else None
        self.find_unused_parameters = find_unused_parameters
        self.require_sync = True
        # sharded update: "auto" shards only on the native engine (with c10d every bucket is all-reduced
        # whole anyway, and the per-region all_gathers would only add collectives), and only once the
        # engine's in-place reduce-scatter / all-gather passed a check on these very ranks
        self.shard_status = None
        if shard_optimizer == "auto":
            shard_optimizer = self.comm is not None
            if shard_optimizer and self.world_size > 1 and self.plan_world == self.world_size:
                ok, why = native_comm.shard_self_test(self.comm, self.process_group)
                self.shard_status = why
                shard_optimizer = ok
        shard_optimizer = bool(shard_optimizer)
        cap = max(1, int(bucket_cap_mb * 1024 * 1024 / 4))
        params = list(store.params)
        # embedding tables exchanged sparsely (parallel/tied.py): out of the buckets; the rest of
        # their module (LayerNorm) is a bucket of its own so that nothing else waits for the
        # embedding backward
        self.tables = None
        own = set()
        if (sparse_embedding is not None and SparseTableSync.supported(store, list(sparse_embedding[0]))
                and SparseTableSync.pays(self.plan_world, sparse_capacity, list(sparse_embedding[0]))):
            tables, rest = sparse_embedding
            self.tables = SparseTableSync(self, list(tables), sparse_capacity)
            own = {id(p) for p in rest}
        skip = {id(p) for p in self.tables.tables} if self.tables is not None else set()
        order = sorted((p for p in params if id(p) not in skip), key=lambda p: store.offset(p), reverse=True)
        self.buckets = []  # (lo, hi, [params])
        if shard_optimizer and store.chunks is not None:
            # sharded update: one bucket per update chunk (embeddings, each layer, the heads), so a
            # chunk's all-gather after the update covers whole buckets
            from hetseq_amd.runtime.flat import bisect_chunk

            per = {}
            for p in order:
                per.setdefault(bisect_chunk(store.chunks, store.offset(p)), []).append(p)
            self.buckets = [per[c] for c in sorted(per, reverse=True)]
            # the layer whose backward finishes last: one bucket per gradient group, each reduced
            # behind its own readiness event from the fused backward (early buckets, below) -- only
            # the last group's reduce-scatter is left for the end of the backward
            eg = getattr(module, "grad_groups", None)
            el = getattr(module, "early_layer", None)
            groups = eg() if callable(eg) and callable(el) and self.comm is not None else None
            if groups:
                ids = [{id(p) for p in g} for g in groups]
                c = bisect_chunk(store.chunks, store.offset(groups[0][0]))
                if c in per and sum(len(x) for x in ids) == len(per[c]) and all(
                        bisect_chunk(store.chunks, store.offset(p)) == c for g in groups for p in g):
                    i = next(k for k, b in enumerate(self.buckets) if b is per[c])
                    subs = [[p for p in per[c] if id(p) in x] for x in ids]
                    self.buckets[i:i + 1] = subs
                    self.early = list(range(i, i + len(subs)))
                    self._early_layer = el()
        else:
            cur, size = [], 0
            for p in order:
                if id(p) in own and cur and not any(id(q) in own for q in cur):
                    self.buckets.append(cur)
                    cur, size = [], 0
                cur.append(p)
                size += p.numel()
                if size >= cap:
                    self.buckets.append(cur)
                    cur, size = [], 0
            if cur:
                self.buckets.append(cur)
        self.ranges = []
        self.bucket_of = {}
        los = sorted(min(store.offset(p) for p in ps) for ps in self.buckets)
        for bi, ps in enumerate(self.buckets):
            lo = min(store.offset(p) for p in ps)
            hi = max(store.offset(p) + p.numel() for p in ps)
            if shard_optimizer and store.chunks is not None:
                # (to the next bucket's start inside its chunk, else the chunk's aligned end: the
                # padding is zero in every buffer, and the region then splits into W whole pieces --
                # runtime/flat.py CHUNK_ALIGN)
                from hetseq_amd.runtime.flat import bisect_chunk

                end = store.chunks[bisect_chunk(store.chunks, lo)][1]
                hi = min([x for x in los if lo < x < end] + [end])
            self.ranges.append((lo, hi))
            for p in ps:
                self.bucket_of[id(p)] = bi
        # a bucket covers [first offset, last end) of its parameters, alignment gaps between them
        # included; gaps between buckets (<= 63 elements of 256-B padding, runtime/flat.py) are in no
        # range: their gradient entries stay zero on every rank and no parameter reads them
        self.shard = None
        if shard_optimizer:
            from hetseq_amd.parallel.zero import ShardPlan

            tables = []
            if self.tables is not None:
                offs = sorted((store.offset(p), store.offset(p) + p.numel()) for p in self.tables.tables)
                for lo, hi in offs:  # contiguous tables (64-element alignment gaps included) as one region
                    if tables and lo - tables[-1][1] < 64:
                        tables[-1] = (tables[-1][0], hi)
                    else:
                        tables.append((lo, hi))
            rank = dist.get_rank(self.process_group) if self.plan_world == self.world_size else 0
            self.shard = ShardPlan(store, self.ranges, tables, self.plan_world, rank, comm=self.comm,
                                   group=self.process_group)
            store.shard = self.shard
        if self.early and self.shard is not None and store.grad.is_cuda:
            import array

            from hetseq_amd.ops._C import hip

            self._early_ev = array.array("q", [hip().event_create() for _ in self.early])
            self._early_layer.__dict__["_hs_early"] = (self._early_ev.buffer_info()[0], self._early_launch)
        else:
            self.early = []
        self._reset_state()
        # Readiness = post-accumulate-grad hooks.  They also fire when a fused
        # Function returned None for a parameter whose gradient it accumulated
        # directly into the flat buffer (the AccumulateGrad node still runs, after
        # that Function's kernels were enqueued), so one signal covers both paths.
        self._hooks = [p.register_post_accumulate_grad_hook(self._grad_ready) for p in params]
        # fused layers whose backward writes the store directly report their parameters here (one
        # call per layer instead of one hook per parameter: models/bert.py BertLayer.fused)
        store.ready_cb = self._params_ready
        if broadcast and (self.world_size > 1 or self.comm is not None):
            with torch.no_grad():
                if self.comm is not None:
                    self.comm.broadcast(store.param, src=0)
                else:
                    dist.broadcast(store.param, src=0, group=self.process_group)
            store.bump()
            store.sync_shadow()

    early = []  # bucket indices reduced behind the fused backward's group events (backward order)

    # The early layer's last group (QKV) is complete only after the weight-gradient stream's last
    # products, ~40 us after the embedding backward's rows are ready; the comm stream runs in issue
    # order, so its reduce-scatter issued first held the rows' all-gather (the step's largest tail
    # collective) behind it.  With the sparse table exchange armed that group is deferred until the
    # rows' all-gather is enqueued (parallel/tied.py rows_ready -> launch_deferred_early).
    DEFER_LAST_EARLY = True

    def _early_launch(self):
        """Right after the early layer's fused backward was enqueued (ops/bert_ops.py): reduce its
        gradient groups, each behind the event the backward recorded when the group was complete."""
        if not self.require_sync:
            return
        defer = self.DEFER_LAST_EARLY and self.tables is not None and self.tables.armed
        for k, b in enumerate(self.early):
            if self.next_launch != b:  # (an earlier bucket is not out yet: the hooks launch in order)
                return
            if defer and k == len(self.early) - 1:
                self._deferred_early = k
                return
            self._launch_early(k)

    def _launch_early(self, k):
        b = self.early[k]
        lo, hi = self.ranges[b]
        self.comm.wait_events([self._early_ev[k]])
        self._launch_range(lo, hi, "reducescatter_group%d" % b, producers=None)
        self.next_launch += 1

    def launch_deferred_early(self):
        """The deferred early group (see DEFER_LAST_EARLY), then any bucket that became ready behind it."""
        k = self._deferred_early
        if k is None:
            return
        self._deferred_early = None
        self._launch_early(k)
        self._launch_ready()

    def _reset_state(self):
        self.pending = [len(ps) for ps in self.buckets]
        self.ready = [False] * len(self.buckets)
        self.next_launch = 0
        self.works = []
        self.callback_queued = False
        # collectives of this step: (what, payload bytes per rank, issued after the last backward
        # kernel, bytes each rank RECEIVES over the links)
        self.comm_log = []
        self._in_tail = False
        self._deferred_early = None

    def _log(self, what, t, kind="allreduce"):
        n = t.numel() * t.element_size()
        W = getattr(self, "plan_world", self.world_size)
        # ring collectives: an all-reduce receives 2(W-1)/W of the payload, an all-gather the other
        # W-1 ranks' payloads
        recv = ((W - 1) * n if kind == "allgather" else (W - 1) * n // max(W, 1) if kind == "reducescatter"
                else 2 * (W - 1) * n // max(W, 1))
        self.comm_log.append((what, n, self._in_tail, recv))

    def _tail_started(self):
        """Called once the last backward Function enqueued its kernels (the embedding backward)."""
        self._in_tail = True

    def tail_bytes(self):
        """Bytes each rank receives in the collectives issued after the last backward kernel (this
        step): what the exposed communication tail has to move over the links."""
        return sum(r for _, _, tail, r in self.comm_log if tail)

    # ------------------------------------------------------------- forward
    def forward(self, *inputs, **kwargs):
        if self.require_sync:
            self._reset_state()
            if self.tables is not None:
                self.tables.reset()
        return self.module(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_sync
        self.require_sync = False
        try:
            yield
        finally:
            self.require_sync = old

    # ------------------------------------------------------------- hooks
    def _params_ready(self, params):
        for p in params:
            self._grad_ready(p)

    def _grad_ready(self, p):
        if not self.require_sync:
            return
        if not self.callback_queued:
            self.callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b = self.bucket_of.get(id(p))
        if b is None:  # a sparsely exchanged table (parallel/tied.py)
            return
        self.pending[b] -= 1
        if self.pending[b] == 0:
            self.ready[b] = True
            self._launch_ready()

    def _launch_ready(self):
        while self.next_launch < len(self.buckets) and self.ready[self.next_launch]:
            if self._deferred_early is not None and self.next_launch == self.early[self._deferred_early]:
                return  # (held back behind the rows' all-gather: launch_deferred_early)
            self._launch(self.next_launch)
            self.next_launch += 1

    def _launch(self, b):
        lo, hi = self.ranges[b]
        if b == len(self.buckets) - 1 and (self.tables is None or not self.tables.armed):
            self._tail_started()  # the last bucket waited for the embedding backward (dense tables)
        self._launch_range(lo, hi, "allreduce_bucket%d" % b)

    def _launch_range(self, lo, hi, name, producers=()):
        profiling.range_push(name)
        self.store.flush_range(lo, hi)  # (a lazily zeroed region no writer claimed: cleared before reducing)
        g = self.store.grad
        rs = self.shard is not None and self.comm is not None and self.shard.by_range[(lo, hi)].ps > 0
        self._log(name, g[lo:hi], "reducescatter" if rs else "allreduce")
        side = streams.active(g.device) if g.is_cuda else None
        if self.comm is not None:
            # the comm stream waits for both producers; neither producer stream is stalled
            cur = torch.cuda.current_stream(g.device)
            prod = None if producers is None else ((cur, side) if side is not None else (cur,))
            if self.shard is not None:  # sharded update: reduce-scatter (tail all-reduced)
                self.shard.reduce_bucket(lo, hi, prod)
            else:
                self.comm.all_reduce_async(g[lo:hi], producers=prod)
            work = None
        elif side is not None:
            # the bucket's weight gradients come from the wgrad side stream, its biases / LN
            # from the compute stream: issue the collective from the side stream after it
            # waits for the compute stream, so RCCL orders after both without stalling compute
            side.wait_stream(torch.cuda.current_stream(g.device))
            with torch.cuda.stream(side):
                work = dist.all_reduce(g[lo:hi], group=self.process_group, async_op=True)
        else:
            work = dist.all_reduce(g[lo:hi], group=self.process_group, async_op=True)
        profiling.range_pop()
        if work is not None:
            self.works.append(work)

    def _finalize(self):
        self.launch_deferred_early()
        if self.next_launch < len(self.buckets):
            missing = [i for i in range(len(self.buckets)) if not self.ready[i]]
            if missing and not self.find_unused_parameters:
                raise RuntimeError(
                    "Expected to have finished reduction in the prior iteration; buckets {} never became ready. "
                    "Pass --find-unused-parameters if some parameters legitimately receive no gradient.".format(
                        missing))
            for i in missing:
                self.ready[i] = True
            self._launch_ready()
        if self.tables is not None:
            self.tables.launch_pending()
        if self.store.grad.is_cuda:
            streams.join()  # compute stream after the wgrad stream (and the collectives issued on it)
        if self.comm is not None:
            self.comm.wait()  # compute stream after the comm stream (no host synchronisation)
            self.comm.check()  # raises if the watchdog aborted a stuck / failed collective
        for w in self.works:
            w.wait()
        self.works = []
        if self.tables is not None:
            self.tables.scatter()  # gathered embedding rows into the reduced tables

    def all_reduce_grads(self):
        """SUM the whole flat gradient buffer across the group in one collective (the split-graph
        path: backward ran without communication, parallel bucket overlap is not available)."""
        g = self.store.grad
        if self.comm is not None and g.is_cuda:
            self.comm.all_reduce(g)
        else:
            dist.all_reduce(g, group=self.process_group)
        return g

    def all_reduce_(self, t):
        """In-place SUM of a small device tensor across the data-parallel group (fast stats)."""
        if self.comm is not None and t.is_cuda:
            return self.comm.all_reduce(t)
        dist.all_reduce(t, group=self.process_group)
        return t

    def parameters(self, recurse=True):
        return self.module.parameters(recurse)

    def named_parameters(self, *a, **k):
        return self.module.named_parameters(*a, **k)

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, *a, **k):
        return self.module.load_state_dict(*a, **k)


class BMUF(object):
    """Blockwise Model-Update Filtering (Chen & Huo 2016) for ``--use-bmuf``.

    Each rank runs its own optimizer; every ``sync_interval`` updates the
    flat parameters are averaged (one all-reduce) and a block-momentum
    filtered global step is applied.  The reference only exposes the flag
    and silently trains ranks independently (Q08).
    """

    def __init__(self, store, process_group=None, block_momentum=0.875, block_lr=1.0, sync_interval=1):
        self.store = store
        self.group = process_group or dist.group.WORLD
        self.world_size = dist.get_world_size(self.group)
        self.bm = block_momentum
        self.blr = block_lr
        self.interval = max(1, sync_interval)
        with torch.no_grad():
            dist.broadcast(store.param, src=0, group=self.group)
        self.global_params = store.param.detach().clone()
        self.smoothed = torch.zeros_like(self.global_params)
        self.count = 0

    @torch.no_grad()
    def after_step(self):
        self.count += 1
        if self.count % self.interval:
            return
        p = self.store.param
        dist.all_reduce(p, group=self.group)
        p.div_(self.world_size)
        delta = self.global_params - p
        self.smoothed.mul_(self.bm).add_(delta, alpha=self.blr)
        self.global_params.sub_(self.smoothed)
        # Nesterov-style look-ahead for the next block
        p.copy_(self.global_params).sub_(self.smoothed, alpha=self.bm)
        self.store.sync_shadow()
