"""Native launch path of the fused encoder layer on the h3p engine (csrc/kernels/layer_prog.cpp).

The Python layer (ops/bert_ops.py ``_layer_forward_h3p`` / ``_layer_backward_h3p``) resolves every
launch per call: output allocation, row-slice views, pointer and stride arguments, ~30 wrapper calls
per layer and step.  A :class:`LayerProgram` resolves them once per layer and batch shape into an
int64 plan (the field names come from the extension, so the two sides cannot drift) over a
persistent ARENA -- the layer's activations, planes, backward scratch -- and the forward and the
backward are one extension call each.  Same kernels, same arguments, same streams and fork points as
the Python layer (tests/test_layer_prog_gpu.py checks bitwise equality).

Arena lifetime: the buffers are rewritten by the next forward of the same layer.  Everything that
reads them is ordered before that by the streams: the backward of a step precedes the next forward
on the compute stream, the side stream's weight-gradient reads precede the next forward's second
half-batch chain (the same stream) and the compute stream waits for the side stream at the end of
every backward (runtime/streams.py ``join``).  The layer output handed to autograd is a fresh view
of the arena (a new tensor object per call).

Eligible: training forwards (autograd recording) of a layer whose gradients go into a flat store
with the side stream enabled, no activation checkpointing, on the h3p engine.  Reference: one
BertLayer forward / backward (bert_modeling.py:361-441).
"""
from __future__ import annotations

import array

import torch

from hetseq_amd.ops import h3p
from hetseq_amd.ops._C import hip

_FIELDS = None
_SLABS: dict = {}  # device -> (numel, slab for the compute stream, slab for the side stream)
_OLD_SLABS: list = []  # smaller pairs earlier programs still address


def fields():
    global _FIELDS
    if _FIELDS is None:
        _FIELDS = {n: i for i, n in enumerate(hip().layer_plan_fields())}
    return _FIELDS


def _slabs(device, n):
    e = _SLABS.get(device)
    if e is None or e[0] < n:
        if e is not None:
            _OLD_SLABS.append(e)
        e = (n, torch.empty(n, dtype=torch.float32, device=device), torch.empty(n, dtype=torch.float32, device=device))
        _SLABS[device] = e
    return e


class LayerProgram(object):
    """Plan and arena of one encoder layer for one batch shape (B, S) and dropout setting."""

    def __init__(self, W, Gv, B, S, NH, halves, ks_wo, ks_w2, ksg, dropout_attn, device):
        from hetseq_amd.ops import bert_ops

        F_ = fields()
        Wp = W.h3p
        H = W.wo.shape[0]
        Fd = W.w1.shape[0]
        rows = B * S
        self.key = (id(Wp), id(Gv), B, S, halves, bool(dropout_attn))
        self.rows, self.H, self.F = rows, H, Fd
        f32 = dict(dtype=torch.float32, device=device)
        z = lambda *shape: torch.empty(shape, **f32)  # noqa: E731
        self.qkv, self.ctx = z(rows, 3 * H), z(rows, H)
        self.lse = z(B * NH * S)
        self.dmask = (torch.empty(B * NH * S * (S // 32), dtype=torch.int32, device=device) if dropout_attn else None)
        self.h1, self.z1, self.h2, self.z2 = (z(rows, H) for _ in range(4))
        self.m1, self.r1, self.m2, self.r2 = (z(rows) for _ in range(4))
        self.f1pre = z(rows, Fd)
        self.ctxp, self.h1p, self.h2p = (h3p.empty(rows, H, device) for _ in range(3))
        self.f1p = h3p.empty(rows, Fd, device)
        self.dz2, self.dz1, self.dctx = z(rows, H), z(rows, H), z(rows, H)
        self.dbuf = z(B * NH * S)  # (dqkv itself exists only as the planes dqkvp)
        self.da2p, self.da1p = h3p.empty(rows, H, device), h3p.empty(rows, H, device)
        self.df1p, self.dqkvp = h3p.empty(rows, Fd, device), h3p.empty(rows, 3 * H, device)
        nb = rows // 4  # (the most column-partial rows any ln_bwd_h3p kernel writes: 4-row workgroups)
        self.part2, self.part1 = bert_ops._colpart_buf(nb, H, device), bert_ops._colpart_buf(nb, H, device)
        self.psync_f, self.psync_b = bert_ops.panel_sync(device, rows, 0), bert_ops.panel_sync(device, rows, 1)
        self.part_gelu = z(rows // 128, Fd)
        self.part_bq = z(rows // 32, 3 * H)  # the QKV bias gradient's column partials (from dqkvp)
        # dS of the attention backward, [B * NH][S queries][S keys] fp32: the dQ product reads it instead of
        # recomputing it (bert_ops._ATTN_DS; None: the fused dQ role)
        self.dsbuf = z(B * NH * S * S) if bert_ops._attn_ds(S) else None
        hr = rows // halves
        need = max(ks_wo * hr * H, ks_w2 * hr * H, ksg["w2"] * H * Fd, ksg["w1"] * Fd * H, ksg["wo"] * H * H,
                   ksg["qkv"] * 3 * H * H)
        n, self.slab0, self.slab1 = _slabs(device, need)
        self.W, self.Gv = W, Gv  # (their storage stays alive with the program)
        q = array.array("q", [0] * len(F_))

        def put(name, v):
            q[F_[name]] = int(v)

        def put_hp(name, hp):
            for k, v in (("p", hp.data_ptr()), ("ld", hp.ld), ("ps", hp.ps), ("e", hp.exps_ptr()), ("lde", hp.lde),
                         ("blk", int(hp.blk))):
                put("%s_%s" % (name, k), v)

        for k, v in (("B", B), ("S", S), ("NH", NH), ("H", H), ("F", Fd), ("rows", rows), ("halves", halves),
                     ("ks_wo", ks_wo), ("ks_w2", ks_w2), ("ksg_qkv", ksg["qkv"]), ("ksg_wo", ksg["wo"]),
                     ("ksg_w1", ksg["w1"]), ("ksg_w2", ksg["w2"]), ("slab_floats", n)):
            put(k, v)
        for k in ("wqkv", "wo", "w1", "w2"):
            put_hp(k, getattr(Wp, k))
        for k in ("bqkv", "bo", "g1", "b1", "bi", "b2", "g2", "bb2"):
            t = getattr(W, k)
            assert t.is_contiguous() and t.dtype == torch.float32
            put(k, t.data_ptr())
        for k in ("qkv", "ctx", "lse", "h1", "z1", "m1", "r1", "f1pre", "h2", "z2", "m2", "r2", "dz2", "dz1", "dctx",
                  "dbuf"):
            put(k, getattr(self, k).data_ptr())
        put("dmask", self.dmask.data_ptr() if self.dmask is not None else 0)
        for k in ("ctxp", "h1p", "f1p", "h2p", "da2p", "df1p", "da1p", "dqkvp"):
            put_hp(k, getattr(self, k))
        put("slab0", self.slab0.data_ptr())
        put("slab1", self.slab1.data_ptr())
        gmap = (("gwqkv", "wqkv"), ("gbqkv", "bqkv"), ("gwo", "wo"), ("gbo", "bo"), ("gg1", "g1"), ("gb1", "b1"),
                ("gw1", "w1"), ("gbi", "bi"), ("gw2", "w2"), ("gb2", "b2"), ("gg2", "g2"), ("gbb2", "bb2"))
        for k, a in gmap:
            t = getattr(Gv, a)
            assert t.is_contiguous() and t.dtype == torch.float32
            put(k, t.data_ptr())
        for i, k in enumerate(("g", "b", "bias")):
            put("part2_" + k, self.part2[i].data_ptr())
            put("part1_" + k, self.part1[i].data_ptr())
        put("part_gelu", self.part_gelu.data_ptr())
        put("psync_f", self.psync_f.data_ptr())
        put("psync_b", self.psync_b.data_ptr())
        put("part_bq", self.part_bq.data_ptr())
        put("dsbuf", self.dsbuf.data_ptr() if self.dsbuf is not None else 0)
        self.q = q
        self.addr = q.buffer_info()[0]
        self._xp = None

    def set_input_layout(self, xp):
        """The layer input's plane layout (the embedding's planes, a split, or the previous layer's)."""
        lay = (xp.ld, xp.ps, xp.lde, int(xp.blk))
        if lay != self._xp:
            F_ = fields()
            for k, v in zip(("xp_ld", "xp_ps", "xp_lde", "xp_blk"), lay):
                self.q[F_[k]] = v
            self._xp = lay
