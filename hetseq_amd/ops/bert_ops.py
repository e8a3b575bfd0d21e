"""Fused BERT operators (autograd Functions over the gfx950 kernels).

Each Function owns a whole sub-graph of the reference model so the
intermediate tensors, kernel fusion and gradient accumulation are under our
control:

* ``FusedEmbedding``   word+pos+type gather -> LN -> dropout   (bert_modeling.py:306-320)
* ``FusedBertLayer``   QKV GEMM -> flash attention -> out-proj -> bias/dropout/residual/LN
                       -> FFN1 -> bias+GELU -> FFN2 -> bias/dropout/residual/LN
                       (bert_modeling.py:323-441), with in-Function activation
                       recomputation for ``--checkpoint-activations``
* ``FusedPreTrainingLoss``  masked-row compaction -> transform(GEMM+GELU+LN) -> tied
                       decoder GEMM on masked rows only -> fused cross-entropy, plus
                       pooler(tanh) -> NSP -> CE -> loss sum in the pool_nsp kernels
                       (bert_modeling.py:506-581, 875-888)
Standalone ops used by tests and other models: ``attention``, ``layer_norm``,
``bias_dropout_residual_ln``, ``bias_gelu``.

All shapes are checked on the host before any launch.  Gradients of
parameters are produced in fp32 (master precision) in both --dtype modes.
"""
from __future__ import annotations

import os

import torch

from hetseq_amd.ops import gemm as G

# the attention-output and FFN-out products' split-K partials summed by the LN forward instead of a
# reduce pass 
_LN_PARTIALS = True
_LN_PARTIALS_WO = _LN_PARTIALS  # (the attention-output product's part of the switch, for bench --ab)
# the QKV bias gradient summed by the QKV weight-gradient kernel (gemm.linear_wgrad_colsum) instead of
# a column-sum pass over dqkv 
_WGRAD_COLSUM = True
# the FFN-in bias gradient the same way, from the FFN-in weight-gradient launch on the side stream,
# instead of the dGELU data-gradient epilogue's column partials + a reduce pass on the compute stream
# 
_FFN_BIAS_WGRAD = True
# the pooler / NSP parameter gradients on the weight-gradient stream
_POOL_WGRAD_SIDE = True
# weight gradients store (beta 0) in the first backward after zero_grad
_FRESH_WGRAD = True
from hetseq_amd.ops._C import dtype_code, hip, stream_handle
from hetseq_amd.parallel import tied
from hetseq_amd.runtime import rng, streams

LN_WIDTHS = (256, 512, 768, 1024, 1536, 2048)


def _err_flag(device):
    """Device-side error word (bit0: embedding id out of range, bit1: MLM overflow, bit2: sort key
    out of range)."""
    key = ("err", device.index)
    buf = _BUFS.get(key)
    if buf is None:
        buf = torch.zeros(1, dtype=torch.int32, device=device)
        _BUFS[key] = buf
    return buf


_BUFS: dict = {}


def check_device_errors(device=None):
    for k, v in list(_BUFS.items()):
        if k[0] == "err" and (device is None or v.device == device):
            e = int(v.item())
            if e & 1:
                raise RuntimeError("embedding lookup got an id outside the vocabulary / type range")
            if e & 2:
                raise RuntimeError("masked-LM rows exceeded the configured capacity (max_predictions_per_seq)")
            if e & 4:
                raise RuntimeError("sort_keys got a key outside [0, bound) (gradient rows would be misplaced)")


def _colpart_buf(nparts, H, device, n=3):
    return torch.empty((n, nparts, H), dtype=torch.float32, device=device)


_PSYNC: dict = {}  # (device, region) -> zero-initialised panel records
_OLD_PSYNC: list = []  # smaller record sets that plans built earlier still address


def panel_sync(device, rows, region):
    """Panel records (csrc/kernels/h3p.h psync_*) for ``rows`` rows of whole-batch row indices: the h3p
    LayerNorm kernels' workgroups exchange their block |max| through them.  ``region`` 0 serves the
    forward (its two half-batch streams address disjoint panels), 1 the backward, 2 the masked-LM
    head's transform LayerNorm.  Zeroed once here;
    the kernels leave every record ready for its next call."""
    key = (device, region)
    t = _PSYNC.get(key)
    need = (rows + 31) // 32 * hip().panel_sync_words()
    if t is None or t.numel() < need:
        if t is not None:
            _OLD_PSYNC.append(t)
        t = torch.zeros(max(need, 128 * hip().panel_sync_words()), dtype=torch.int32, device=device)
        _PSYNC[key] = t
    return t


def ln_bwd_h3p_parts(rows):
    """Column-partial rows of ln_bwd_h3p (one per 8-row workgroup)."""
    return rows // hip().ln_bwd_h3p_part_rows(1)


# --------------------------------------------------------------------- basic ops
def ln_fwd(a, gamma, beta, eps=1e-12, bias=None, resid=None, p=0.0, mode=0, seed=0, off=0, save_z=True,
           outs=None, row0=0, amax=None):
    """LayerNorm forward (+ bias / dropout / residual in mode 1).
    ``a`` may be [ks, rows, H] split-K partials of the producing GEMM (gemm.linear_fwd_partials),
    summed in slice order as the GEMM's own reduce pass would.  ``outs`` = (y, z, mean, rstd) buffers to
    write (row slices of whole-batch tensors); ``row0``: the first row's index in the whole batch
    (the dropout mask is drawn by whole-batch element index, as the backward regenerates it).
    ``amax``: a 1-element slot (ops.gemm.AmaxPool) the kernel atomically maxes |y| into (the h3
    GEMM engine's operand scale for the next product)."""
    nslab = 1
    if a.dim() == 3:
        nslab = a.shape[0]
        stride = a.stride(0)
        a = a[0]
    rows, H = a.shape
    assert H in LN_WIDTHS and a.is_contiguous() and (resid is None or resid.shape == a.shape)
    if outs is not None:
        y, z, mean, rstd = outs
    else:
        y = torch.empty_like(a)
        z = torch.empty((rows, H), dtype=torch.float32, device=a.device) if save_z else None
        mean = torch.empty(rows, dtype=torch.float32, device=a.device)
        rstd = torch.empty_like(mean)
    hip().ln_fwd(dtype_code(a), a.data_ptr(), bias.data_ptr() if bias is not None else 0,
                 resid.data_ptr() if resid is not None else 0, gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                 z.data_ptr() if z is not None else 0, mean.data_ptr(), rstd.data_ptr(), rows, H, float(eps), float(p),
                 seed, off, mode, stream_handle(), nslab, stride if nslab > 1 else 0, int(row0),
                 G.slot_ptr(amax))
    return y, z, mean, rstd


def ln_fwd_h3p(a, gamma, beta, eps, bias, resid, p, seed, off, outs, row0, hp, amax=None, region=0):
    """ln_fwd (bias-dropout-residual mode, fp32) that also writes y as h3p planes into ``hp`` (an
    ops.h3p.HP over the same rows): the next product's operand without a split pass.  ``region``: the
    panel records (panel_sync) -- 0 the encoder's forward, 2 the masked-LM head's transform."""
    assert hp.blk, "producers write blocked planes"
    nslab, stride = 1, 0
    if a.dim() == 3:
        nslab, stride = a.shape[0], a.stride(0)
        a = a[0]
    rows, H = a.shape
    y, z, mean, rstd = outs
    psync = panel_sync(a.device, int(row0) + rows, region)
    hip().ln_fwd_h3p(a.data_ptr(), bias.data_ptr() if bias is not None else 0,
                     resid.data_ptr() if resid is not None else 0, gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                     z.data_ptr(), mean.data_ptr(), rstd.data_ptr(), rows, H, float(eps), float(p), seed, off, 1,
                     nslab, stride, int(row0), G.slot_ptr(amax), hp.data_ptr(), hp.ps, hp.exps_ptr(),
                     psync.data_ptr(), int(row0) // 32, stream_handle())
    return y


def ln_bwd_h3p(dy, z, mean, rstd, gamma, p, seed, off, hp, acc=None, side=False):
    """LN backward of the bias-dropout-residual LN: dz (fp32, returned) and da written only as h3p
    planes into ``hp``; parameter gradients (dgamma, dbeta, dbias) accumulated into ``acc`` (flat-store
    views; finalised on the weight-gradient stream with ``side``) or returned fresh."""
    assert hp.blk, "producers write blocked planes"
    rows, H = dy.shape
    nb = ln_bwd_h3p_parts(rows)
    part = _colpart_buf(nb, H, dy.device)
    dz = torch.empty_like(dy)
    psync = panel_sync(dy.device, rows, 1)
    hip().ln_bwd_h3p(dy.data_ptr(), z.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(), dz.data_ptr(),
                     part[0].data_ptr(), part[1].data_ptr(), part[2].data_ptr(), rows, H, float(p), seed, off,
                     hp.data_ptr(), hp.ps, hp.exps_ptr(), psync.data_ptr(), stream_handle())
    if acc is not None:
        outs = list(acc[:3])

        def fin():
            hip().colpart_finalize([part[i].data_ptr() for i in range(3)], [o.data_ptr() for o in outs], nb, H, 1,
                                   stream_handle())
        if side:
            streams.run(dy.device, fin, part)
        else:
            fin()
    else:
        outs = torch.empty((3, H), dtype=torch.float32, device=dy.device)
        hip().colpart_finalize([part[i].data_ptr() for i in range(3)], [outs[i].data_ptr() for i in range(3)], nb, H,
                               0, stream_handle())
    return dz, outs[0], outs[1], outs[2]


def ln_bwd(dy, z, mean, rstd, gamma, p=0.0, mode=0, seed=0, off=0, want_dz=True, want_da=False, dz_out=None,
           acc=None, side=False, amax=None):
    """LN backward.  ``acc`` = (dgamma, dbeta[, dbias]) fp32 tensors to ACCUMULATE into
    (flat-store gradient views); otherwise fresh tensors are returned.  ``side``: run the
    parameter-gradient finalisation on the weight-gradient stream (runtime/streams.py) --
    only dz / da are on the critical path.
    ``amax``: slot receiving |max| of da (mode 1) or dz (mode 0) -- the next GEMMs' operand."""
    rows, H = dy.shape
    nb = hip().ln_bwd_num_blocks()
    part = _colpart_buf(nb, H, dy.device)
    dz = (dz_out if dz_out is not None else torch.empty_like(dy)) if want_dz else None
    da = torch.empty_like(dy) if want_da else None
    hip().ln_bwd(dtype_code(dy), dy.data_ptr(), z.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(),
                 dz.data_ptr() if dz is not None else 0, da.data_ptr() if da is not None else 0, part[0].data_ptr(),
                 part[1].data_ptr(), part[2].data_ptr(), rows, H, float(p), seed, off, mode, stream_handle(),
                 G.slot_ptr(amax))
    n = 3 if mode == 1 else 2
    if acc is not None:
        outs = list(acc[:n])
        assert all(o.is_contiguous() and o.dtype == torch.float32 for o in outs)

        def fin():
            hip().colpart_finalize([part[i].data_ptr() for i in range(n)], [o.data_ptr() for o in outs], nb, H, 1,
                                   stream_handle())

        if side:
            streams.run(dy.device, fin, part)
        else:
            fin()
    else:
        outs = torch.empty((n, H), dtype=torch.float32, device=dy.device)
        hip().colpart_finalize([part[i].data_ptr() for i in range(n)], [outs[i].data_ptr() for i in range(n)], nb, H,
                               0, stream_handle())
    dgamma, dbeta = outs[0], outs[1]
    dbias = outs[2] if mode == 1 else None
    return dz, da, dgamma, dbeta, dbias


def bias_gelu_fwd(x, b, out=None):
    y = torch.empty_like(x) if out is None else out
    rows, N = x.shape
    assert N % 4 == 0 and x.is_contiguous()
    hip().bias_gelu_fwd(dtype_code(x), x.data_ptr(), b.data_ptr(), y.data_ptr(), rows, N, stream_handle())
    return y


def gelu_bwd_colsum(dy, x, b, db_acc=None, amax=None):
    """dx = dy * gelu'(x+b) and db = sum_rows(dx) (accumulated into ``db_acc`` if given); ``amax``: a
    zeroed |max| slot the kernel maxes |dx| into."""
    rows, N = dy.shape
    assert N % 4 == 0 and dy.is_contiguous() and x.is_contiguous()
    chunks = hip().colsum_row_chunks(rows)
    part = torch.empty((chunks, N), dtype=torch.float32, device=dy.device)
    db = db_acc if db_acc is not None else torch.empty(N, dtype=torch.float32, device=dy.device)
    dx = torch.empty_like(dy)
    hip().colsum(dtype_code(dy), dy.data_ptr(), x.data_ptr(), b.data_ptr(), dx.data_ptr(), part.data_ptr(),
                 db.data_ptr(), rows, N, 1 if db_acc is not None else 0, stream_handle(), amax=G.slot_ptr(amax))
    return dx, db


def colsum(x, acc=None):
    """Column sums of x (fp32), accumulated into ``acc`` if given."""
    rows, N = x.shape
    assert x.is_contiguous()
    chunks = hip().colsum_row_chunks(rows)
    part = torch.empty((chunks, N), dtype=torch.float32, device=x.device)
    out = acc if acc is not None else torch.empty(N, dtype=torch.float32, device=x.device)
    hip().colsum(dtype_code(x), x.data_ptr(), 0, 0, 0, part.data_ptr(), out.data_ptr(), rows, N,
                 1 if acc is not None else 0, stream_handle())
    return out


def attn_fwd(qkv, mask, B, S, NH, p, seed, off, bias=None, outs=None, b0=0, amax=None):
    """qkv [B*S, 3H] (un-biased projection output if ``bias`` [3H] fp32 is given).  ``outs`` =
    (ctx, lse, dmask) buffers to write (slices of whole-batch tensors); ``b0``: the slice's first
    sequence in the whole batch (its dropout keep bits are the whole-batch launch's).  ``amax``:
    slot receiving |max| of ctx (written by the h3 kernel itself, else one pass behind it)."""
    T, H3 = qkv.shape
    H = H3 // 3
    assert T == B * S and H == NH * 64 and S % 32 == 0 and qkv.is_contiguous()
    assert mask.dtype == torch.int64 and mask.shape == (B, S) and mask.is_contiguous()
    assert bias is None or (bias.shape == (H3,) and bias.dtype == torch.float32 and bias.is_contiguous())
    if outs is not None:
        ctx, lse, dmask = outs
    else:
        ctx = torch.empty((T, H), dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty((B * NH * S,), dtype=torch.float32, device=qkv.device)
        # 1 keep-bit per attention probability, packed 32 keys per word, for the backward
        dmask = torch.empty((B * NH * S * (S // 32),), dtype=torch.int32, device=qkv.device) if p > 0 else None
    done = hip().attn_fwd(dtype_code(qkv), qkv.data_ptr(), mask.data_ptr(), bias.data_ptr() if bias is not None else 0,
                          ctx.data_ptr(), lse.data_ptr(), dmask.data_ptr() if dmask is not None else 0, B, S, NH, 64,
                          float(p), seed, off, stream_handle(), int(b0) * NH,
                          G.slot_ptr(amax) if amax is not None else 0)
    if amax is not None and not done:  # (engines other than h3: one |max| pass behind the kernel)
        G.amax_into(ctx, amax)
    return ctx, (lse, dmask)


def attn_bwd(qkv, mask, ctx, dctx, lse, B, S, NH, p, seed=0, off=0, bias=None, amax=None):
    """``lse`` is the (lse, dropout-bitmask) pair returned by :func:`attn_fwd`; ``amax``: slot
    receiving |max| of dqkv."""
    lse, dmask = lse
    assert dctx.is_contiguous() and dctx.shape == ctx.shape
    assert p == 0 or dmask is not None
    dqkv = torch.empty_like(qkv)
    dbuf = torch.empty_like(lse)
    done = hip().attn_bwd(dtype_code(qkv), qkv.data_ptr(), mask.data_ptr(), bias.data_ptr() if bias is not None else 0,
                          ctx.data_ptr(), dctx.data_ptr(), lse.data_ptr(), dbuf.data_ptr(), dqkv.data_ptr(),
                          dmask.data_ptr() if dmask is not None else 0, B, S, NH, 64, float(p), stream_handle(),
                          G.slot_ptr(amax) if amax is not None else 0)
    if amax is not None and not done:
        G.amax_into(dqkv, amax)
    return dqkv


def attn_fwd_h3p(qkv, mask, B, S, NH, p, seed, off, bias, outs, b0, hp):
    """attn_fwd on the h3 attention kernel that also writes ctx as h3p planes into ``hp`` (an
    ops.h3p.HP over the same rows): the output projection's operand without a split pass."""
    assert hp.blk, "producers write blocked planes"
    ctx, lse, dmask = outs
    hip().attn_fwd_h3p(qkv.data_ptr(), mask.data_ptr(), bias.data_ptr() if bias is not None else 0, ctx.data_ptr(),
                       lse.data_ptr(), dmask.data_ptr() if dmask is not None else 0, B, S, NH, float(p), seed, off,
                       int(b0) * NH, hp.data_ptr(), hp.ps, hp.exps_ptr(), stream_handle())
    return ctx


def attn_bwd_h3p(qkv, mask, ctx, dctx, lse, B, S, NH, p, bias, hp, fp32=True, ds=False):
    """attn_bwd on the h3 attention kernel that also writes dqkv as h3p planes into ``hp``; with
    ``fp32=False`` ONLY as the planes (returns None).  ``ds``: dQ from the stored dS (a B*NH*S*S
    buffer) instead of the fused dQ role."""
    assert hp.blk, "producers write blocked planes"
    lse, dmask = lse
    dqkv = torch.empty_like(qkv) if fp32 else None
    dbuf = torch.empty_like(lse)
    dsb = torch.empty(B * NH * S * S, dtype=torch.float32, device=qkv.device) if ds else None
    hip().attn_bwd_h3p(qkv.data_ptr(), mask.data_ptr(), bias.data_ptr() if bias is not None else 0, ctx.data_ptr(),
                       dctx.data_ptr(), lse.data_ptr(), dbuf.data_ptr(), dqkv.data_ptr() if fp32 else 0,
                       dmask.data_ptr() if dmask is not None else 0, B, S, NH, float(p), hp.data_ptr(), hp.ps,
                       hp.exps_ptr(), stream_handle(), dsbuf=dsb.data_ptr() if dsb is not None else 0)
    return dqkv


def h3p_colpart(hp, part):
    """part[r / 32, c] = column sums of a blocked h3p operand over each 32-row panel (fp32 [rows / 32, cols])."""
    assert hp.blk and part.is_contiguous() and tuple(part.shape) == (hp.rows // 32, hp.cols)
    hip().h3p_colpart(hp.data_ptr(), hp.ld, hp.ps, hp.exps_ptr(), hp.lde, hp.rows, hp.cols, part.data_ptr(),
                      stream_handle())
    return part


# --------------------------------------------------------------------- standalone autograd ops
class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, mask, B, S, NH, p):
        seed, off = rng.fork() if p > 0 else (0, 0)
        out, (lse, dmask) = attn_fwd(qkv.contiguous(), mask, B, S, NH, p, seed, off)
        ctx.save_for_backward(qkv, mask, out, lse, dmask)
        ctx.cfg = (B, S, NH, p, seed, off)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, mask, out, lse, dmask = ctx.saved_tensors
        B, S, NH, p, seed, off = ctx.cfg
        return attn_bwd(qkv, mask, out, dout.contiguous(), (lse, dmask), B, S, NH, p), None, None, None, None, None


def attention(qkv, mask, B, S, NH, p=0.0):
    """Fused BERT attention: qkv [B*S, 3H] -> context [B*S, H]."""
    return _Attention.apply(qkv, mask, B, S, NH, p)


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, bias, resid, p, mode):
        seed, off = rng.fork() if p > 0 else (0, 0)
        y, z, mean, rstd = ln_fwd(x.contiguous(), gamma, beta, eps, bias, resid, p, mode, seed, off)
        ctx.save_for_backward(z, mean, rstd, gamma)
        ctx.cfg = (p, mode, seed, off, bias is not None, resid is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        z, mean, rstd, gamma = ctx.saved_tensors
        p, mode, seed, off, has_bias, has_res = ctx.cfg
        dz, da, dg, db, dbias = ln_bwd(dy.contiguous(), z, mean, rstd, gamma, p, mode, seed, off, True, mode == 1)
        dx = da if mode == 1 else dz
        if mode == 0 and has_bias:
            dbias = dx.float().sum(0)
        return dx, dg, db, None, dbias if has_bias else None, dz if has_res else None, None, None


def layer_norm(x, gamma, beta, eps=1e-12):
    return _LayerNorm.apply(x, gamma, beta, eps, None, None, 0.0, 0)


def bias_dropout_residual_ln(a, bias, resid, gamma, beta, p=0.0, eps=1e-12):
    """LN(dropout(a + bias) + resid) (reference: BertSelfOutput / BertOutput)."""
    return _LayerNorm.apply(a, gamma, beta, eps, bias, resid, p, 1)


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        x = x.contiguous()
        ctx.save_for_backward(x, b)
        return bias_gelu_fwd(x, b)

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        dx, db = gelu_bwd_colsum(dy.contiguous(), x, b)
        return dx, db


def bias_gelu(x, b):
    return _BiasGelu.apply(x, b)


# --------------------------------------------------------------------- embeddings
def segsum_rows(src, order, keys, dst, scratch=None):
    """dst[keys[j]] += src[order[j]] for sorted ``keys`` (deterministic run-wise sums; fp32 src/dst).
    Keys outside [0, dst rows) are skipped; there may be more keys than source rows (one row summed
    into several tables of a concatenated region).  ``scratch``: >= [keys, H] fp32 (run pieces)."""
    H = src.shape[1]
    n = keys.numel()
    assert src.dtype == torch.float32 and dst.dtype == torch.float32 and dst.is_contiguous() and src.is_contiguous()
    assert order.numel() == n and dst.shape[1] == H
    if scratch is None:
        scratch = torch.empty((n, H), dtype=torch.float32, device=src.device)
    assert scratch.numel() >= n * H and scratch.dtype == torch.float32
    hip().segsum_rows(src.data_ptr(), order.data_ptr(), keys.data_ptr(), scratch.data_ptr(), dst.data_ptr(), n, H,
                      dst.shape[0], stream_handle())
    return dst


def sort_keys(keys, bound):
    """Stable ascending sort of int64 ``keys`` in [0, bound): (sorted keys, source indices), by the
    one-block LDS sort (elementwise.hip sort_keys_kernel); sizes it does not serve (n > 16384 or
    too many key + index bits) use torch.sort(stable=True), which returns the same pair."""
    keys = keys.contiguous().view(-1)
    n = keys.numel()
    out_k = torch.empty_like(keys)
    out_o = torch.empty_like(keys)
    err = _err_flag(keys.device)  # bit 2: a key outside [0, bound) (sorted as clamped; raised by check_device_errors)
    if hip().sort_keys(keys.data_ptr(), n, int(bound), out_k.data_ptr(), out_o.data_ptr(), err.data_ptr(),
                       stream_handle()) == 0:
        return out_k, out_o
    return torch.sort(keys, stable=True)


class FusedEmbedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, wword, wpos, wtype, gamma, beta, p, eps, out_dtype, sink=None, amax=None):
        B, S = ids.shape
        V, H = wword.shape
        TV = wtype.shape[0]
        assert H in LN_WIDTHS and S <= wpos.shape[0] and ids.dtype == torch.int64
        ids = ids.contiguous()
        tt = tt.contiguous() if tt is not None else None
        rows = B * S
        y = torch.empty((rows, H), dtype=out_dtype, device=ids.device)
        z = torch.empty((rows, H), dtype=torch.float32, device=ids.device)
        mean = torch.empty(rows, dtype=torch.float32, device=ids.device)
        rstd = torch.empty_like(mean)
        seed, off = rng.fork() if p > 0 else (0, 0)
        err = _err_flag(ids.device)
        hip().emb_fwd(dtype_code(y), ids.data_ptr(), tt.data_ptr() if tt is not None else 0, wword.data_ptr(),
                      wpos.data_ptr(), wtype.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(), z.data_ptr(),
                      mean.data_ptr(), rstd.data_ptr(), rows, S, H, V, TV, float(eps), float(p), seed, off,
                      err.data_ptr(), stream_handle(), G.slot_ptr(amax))
        ctx.save_for_backward(ids, tt if tt is not None else ids.new_zeros(0), z, mean, rstd, gamma)
        ctx.cfg = (B, S, V, H, TV, wpos.shape[0], p, seed, off, tt is not None)
        ctx.sink = sink
        # data-parallel sparse exchange of the tables' rows (parallel/tied.py): keys gathered now
        ctx.tables = None
        if sink is not None and tied._HANDLERS:
            h = tied.lookup(sink["views"]()[0])
            if h is not None and h.begin(ids, tt, bool(ctx.needs_input_grad[2])):
                ctx.tables = h
        return y

    @staticmethod
    def backward(ctx, dy):
        ids, tt, z, mean, rstd, gamma = ctx.saved_tensors
        B, S, V, H, TV, P, p, seed, off, has_tt = ctx.cfg
        dy = dy.contiguous()
        dev = dy.device
        sink = ctx.sink
        tables = ctx.tables  # rows exchanged by the data-parallel engine: no local table updates
        if sink is not None:  # accumulate straight into the flat gradient buffer
            dword, dpos, dtype_, dg, db = sink["views"]()
            if tables is None:
                streams.wait_mark(dev, "tied")  # the tied decoder's weight GEMM (side stream) also writes dword
        else:
            dword = torch.zeros((V, H), dtype=torch.float32, device=dev)
            dpos = torch.zeros((P, H), dtype=torch.float32, device=dev)
            dtype_ = torch.zeros((TV, H), dtype=torch.float32, device=dev)
            outs = torch.empty((2, H), dtype=torch.float32, device=dev)
            dg, db = outs[0], outs[1]
        nb = hip().ln_bwd_num_blocks()
        part = _colpart_buf(nb, H, dev, 2)
        rows = B * S
        dx = tables.row_buffer(rows, H) if tables is not None else torch.empty((rows, H), dtype=torch.float32,
                                                                                device=dev)
        small_tv = TV <= 2  # token types reduced in-kernel (per-block partials); otherwise by sorted runs
        ptype = _colpart_buf(nb, H, dev, 2) if (small_tv and tables is None) else None
        hip().emb_bwd(dtype_code(dy), dy.data_ptr(), z.data_ptr(), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(),
                      dx.data_ptr(), part[0].data_ptr(), part[1].data_ptr(),
                      tt.data_ptr() if (has_tt and ptype is not None) else 0,
                      ptype.data_ptr() if ptype is not None else 0, rows, H, float(p), seed, off, stream_handle())
        acc = 1 if sink is not None else 0
        hip().colpart_finalize([part[0].data_ptr(), part[1].data_ptr()], [dg.data_ptr(), db.data_ptr()], nb, H, acc,
                               stream_handle())
        if tables is not None:
            tables.rows_ready()  # word / position / type rows: gathered and summed after the exchange
            return (None,) * 12
        if small_tv:
            tv = [ptype[0].data_ptr()] + ([ptype[1].data_ptr()] if TV == 2 else [])
            hip().colpart_finalize(tv, [dtype_[i].data_ptr() for i in range(len(tv))], nb, H, 1, stream_handle())
        else:
            tt_keys, tt_order = sort_keys(tt, TV)
            segsum_rows(dx, tt_order, tt_keys, dtype_)
        # word rows: deterministic sorted-run sums; positions: fixed-order column sums
        word_keys, word_order = sort_keys(ids, V)
        segsum_rows(dx, word_order, word_keys, dword)
        hip().pos_grad(dx.data_ptr(), dpos.data_ptr(), B, S, H, stream_handle())
        if sink is not None:
            return (None,) * 12
        return None, None, dword, dpos, dtype_, dg, db, None, None, None, None, None


# --------------------------------------------------------------------- encoder layer
class LayerWeights(object):
    """Compute views of one encoder layer's weights: fp32 master or bf16 shadow; ``h3p``: the GEMM
    weights' block-scaled planes (ops.h3p.HP) when the layer runs on the h3p engine."""

    __slots__ = ("wqkv", "bqkv", "wo", "bo", "g1", "b1", "w1", "bi", "w2", "b2", "g2", "bb2", "h3p")


class LayerAmax(object):
    """The h3 GEMM engine's |max| slots for one encoder layer (in a forward's ops.gemm.AmaxPool):
    ``w`` = (wqkv, wo, w1, w2) weight slots; ``x`` = the input's slot per half-batch chain (both
    halves read the embedding's one slot in layer 0), ``xw`` = the input's whole-batch partials;
    activation slots at ``base`` + 0 h1, 2 ctx, 4 f1, 6 h2 (one per half each; the un-split
    forward uses the first) and the backward's 8 do, 9 df1, 10 da1, 11 dqkv."""

    NS = 12
    __slots__ = ("pool", "w", "x", "xw", "base")

    def a(self, off, n=1):
        return self.pool.act(self.base + off, n)


def _am(am, *pairs):
    """(A's, B's) slots for a GEMM when ``am`` is set (None: the GEMM wrapper measures the operands)."""
    return None if am is None else pairs


# The fp32 encoder-layer forward runs the batch as two half-batch chains on two streams (the compute
# stream and streams.fwd2, the idle weight-gradient stream): a single chain leaves the GEMMs' last partial round of tiles on a mostly
# idle chip (QKV: 576 tiles of 128 x 128 for 512 block slots), and the other half's kernels fill it
# (12 BERT-base layers 4.96 -> 4.42 ms, tools/fwd_split_probe.py).
_FWD_SPLIT = True
# K split of the half-batch chains' plain GEMMs (None: the per-shape isolated measurement)
_FWD_KS = None


# bf16 compute: the same two half-batch chains (bench.py --ab fsplit_bf16_on / fsplit_bf16_off)
_FWD_SPLIT_BF16 = True


def _fwd_split_ok(x, mask, W, cfg):
    B, S = cfg[0], cfg[1]
    dt_ok = x.dtype == torch.float32 or (x.dtype == torch.bfloat16 and _FWD_SPLIT_BF16)
    return (_FWD_SPLIT and x.is_cuda and dt_ok
            and B % 2 == 0 and B * S >= 1024 and streams.enabled() and x.is_contiguous())


def _layer_forward_split(x, mask, W, cfg, save, am=None):
    """_layer_forward with the batch in two halves on two streams, every op writing its half of the
    whole-batch tensors (the backward sees the same saved tensors as an unsplit forward).  Dropout is
    drawn by whole-batch index (LN: ``row0``, attention: ``b0``): the same masks as one chain."""
    B, S, NH, p_h, p_a, eps, seeds = cfg
    (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
    rows, H = x.shape
    F = W.w1.shape[0]
    dev, f32, dt = x.device, torch.float32, x.dtype  # activations in the compute dtype, statistics fp32
    qkv = torch.empty((rows, 3 * H), dtype=dt, device=dev)
    ctx_ = torch.empty((rows, H), dtype=dt, device=dev)
    lse = torch.empty((B * NH * S,), dtype=f32, device=dev)
    dmask = torch.empty((B * NH * S * (S // 32),), dtype=torch.int32, device=dev) if p_a > 0 else None
    h1, h2 = (torch.empty((rows, H), dtype=dt, device=dev) for _ in range(2))
    z1, z2 = (torch.empty((rows, H), dtype=f32, device=dev) for _ in range(2))
    m1, r1, m2, r2 = (torch.empty((rows,), dtype=f32, device=dev) for _ in range(4))
    f1, f1pre = torch.empty((rows, F), dtype=dt, device=dev), torch.empty((rows, F), dtype=dt, device=dev)
    hr, hb = rows // 2, B // 2
    nl, nm = hb * NH * S, hb * NH * S * (S // 32)
    with streams.fwd_halves(dev) as halves:
        for h in halves:
            r = slice(h * hr, (h + 1) * hr)
            xh = x[r]
            sl = (lambda off: am.a(off + h)) if am is not None else (lambda off: None)  # this half's slot
            G.linear_fwd(xh, W.wqkv, out=qkv[r], ksplit=_FWD_KS, amax=_am(am, am and am.x[h], am and am.w[0]))
            attn_fwd(qkv[r], mask[h * hb:(h + 1) * hb], hb, S, NH, p_a, s_a, o_a, bias=W.bqkv, b0=h * hb,
                     outs=(ctx_[r], lse[h * nl:(h + 1) * nl], dmask[h * nm:(h + 1) * nm] if dmask is not None else None),
                     amax=sl(2))
            wo_am = _am(am, sl(2), am and am.w[1])
            a = (G.linear_fwd_partials(ctx_[r], W.wo, ksplit=_FWD_KS, amax=wo_am)[0] if _LN_PARTIALS_WO
                 else G.linear_fwd(ctx_[r], W.wo, ksplit=_FWD_KS, amax=wo_am))
            ln_fwd(a, W.g1, W.b1, eps, bias=W.bo, resid=xh, p=p_h, mode=1, seed=s_1, off=o_1, row0=h * hr,
                   outs=(h1[r], z1[r], m1[r], r1[r]), amax=sl(0))
            G.linear_gelu_fwd(h1[r], W.w1, W.bi, out=(f1[r], f1pre[r]), amax=_am(am, sl(0), am and am.w[2]),
                              amax_out=sl(4))
            w2_am = _am(am, sl(4), am and am.w[3])
            o = (G.linear_fwd_partials(f1[r], W.w2, ksplit=_FWD_KS, amax=w2_am)[0] if _LN_PARTIALS
                 else G.linear_fwd(f1[r], W.w2, ksplit=_FWD_KS, amax=w2_am))
            ln_fwd(o, W.g2, W.bb2, eps, bias=W.b2, resid=h1[r], p=p_h, mode=1, seed=s_2, off=o_2, row0=h * hr,
                   outs=(h2[r], z2[r], m2[r], r2[r]), amax=sl(6))
    # (inside a fwd_chain the second half may still read these after the return)
    streams.chain_keep(x, mask, qkv, ctx_, lse, dmask, h1, z1, m1, r1, f1, f1pre, h2, z2, m2, r2)
    if save:
        return h2, (qkv, ctx_, lse, dmask, z1, m1, r1, h1, f1pre, f1, z2, m2, r2, x, ctx_)
    return h2, None


def _layer_forward(x, mask, W, cfg, save, am=None, meta=None):
    """One layer forward: the h3p engine's (``W.h3p``), the two half-batch chains (_fwd_split_ok), or
    one chain on the fp32 in-kernel-split / bf16 engines (``am``: the h3 engine's |max| slots)."""
    if getattr(W, "h3p", None) is not None:
        return _layer_forward_h3p(x, mask, W, cfg, save, am, meta)
    if _fwd_split_ok(x, mask, W, cfg):
        return _layer_forward_split(x, mask, W, cfg, save, am)
    streams.chain_join(x.device)  # one chain from here: the half-batch chains meet first
    B, S, NH, p_h, p_a, eps, seeds = cfg
    (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
    sl = (lambda off: am.a(off)) if am is not None else (lambda off: None)  # one chain: the first slot
    qkv = G.linear_fwd(x, W.wqkv, amax=_am(am, am and am.xw, am and am.w[0]))  # bias folded into the attention
    ctx_, (lse, dmask) = attn_fwd(qkv, mask, B, S, NH, p_a, s_a, o_a, bias=W.bqkv, amax=sl(2))
    wo_am = _am(am, sl(2), am and am.w[1])
    a = G.linear_fwd(ctx_, W.wo, amax=wo_am) if not _LN_PARTIALS_WO else G.linear_fwd_partials(
        ctx_, W.wo, amax=wo_am)[0]
    h1, z1, m1, r1 = ln_fwd(a, W.g1, W.b1, eps, bias=W.bo, resid=x, p=p_h, mode=1, seed=s_1, off=o_1, amax=sl(0))
    f1, f1pre = G.linear_gelu_fwd(h1, W.w1, W.bi, amax=_am(am, sl(0), am and am.w[2]),
                                  amax_out=sl(4))  # f1pre: un-biased pre-activation
    # FFN-out product: its split-K partials go straight into the LN (no reduce pass)
    w2_am = _am(am, sl(4), am and am.w[3])
    o = G.linear_fwd(f1, W.w2, amax=w2_am) if not _LN_PARTIALS else G.linear_fwd_partials(f1, W.w2,
                                                                                        amax=w2_am)[0]
    h2, z2, m2, r2 = ln_fwd(o, W.g2, W.bb2, eps, bias=W.b2, resid=h1, p=p_h, mode=1, seed=s_2, off=o_2, amax=sl(6))
    if save:
        return h2, (qkv, ctx_, lse, dmask, z1, m1, r1, h1, f1pre, f1, z2, m2, r2, x, ctx_)
    return h2, None


# ----------------------------------------------------------------- encoder layer on the h3p engine
# fp32 products as three fp16 MFMA products over block-scaled split planes written once per tensor
# (ops/h3p.py, csrc/kernels/gemm_h3p.hip).  K slices of the forward's two N = 768 products, whose
# tile grids (48-96 tiles per half-batch chain) would leave most of the chip idle; their slabs go
# straight into the LayerNorm forward (no reduce pass).
_H3P_KS_WO = 2
_H3P_KS_W2 = 4


class _OneChain(object):
    """The single-chain stand-in for streams.fwd_halves (a batch too small to split)."""

    def __enter__(self):
        return iter((0,))

    def __exit__(self, *exc):
        return False


# the native launch path (ops/layer_prog.py): False runs the Python layer (A/B, bench --ab prog_off)
LAYER_PROG = True
# the second half-batch chain's start in the first layer (layer_prog.cpp layer_fwd_h3p stagger):
# 0 with the first chain, 1 / 2 / 3 after its QKV product / attention / first LayerNorm
_FWD_STAGGER = 0
# the layer program's attention backward: dQ from the dS its dK / dV blocks store (attention_h3.hip
# attn_dq_ds_kernel) instead of the fused dQ role recomputing it, up to _ATTN_DS_MAX_S (bench.py --ab
# attds_on / attds_off: S 128 10.302 -> 10.200 ms; S 512 11.687 -> 11.880, the 100 MB dS round trip
# costs more than the recomputation saves there)
_ATTN_DS = True
_ATTN_DS_MAX_S = 128


def _attn_ds(S):
    return _ATTN_DS and S <= _ATTN_DS_MAX_S
PROG_BUILDS = [0]  # programs built in this process (tests)
_PROG_SIDE_DELAY = 0  # GPU cycles the side stream sleeps before a program backward (tests only)


class _ProgSaved(object):
    """What a program forward leaves for its backward: the program and the input's planes."""
    __slots__ = ("prog", "xp")

    def __init__(self, prog, xp):
        self.prog, self.xp = prog, xp


def _program(W, meta, B, S, NH, p_a, halves, dev):
    """The layer's :class:`~hetseq_amd.ops.layer_prog.LayerProgram` for this shape, or None when the
    forward is not eligible (no flat store / side stream, recompute; ``meta`` None: no backward)."""
    if not (LAYER_PROG and not meta.get("recompute") and streams.enabled()
            and meta.get("grad_sink") is not None and meta.get("store") is not None):
        return None
    Gv = meta["grad_sink"]()
    # (held by the layer module: a program -- its arena, the store addresses it bakes in -- lives as
    # long as the model it was built for)
    progs = meta["weights"].__self__.__dict__.setdefault("_hs_progs", {})
    key = (id(W.h3p), id(Gv), B, S, halves, p_a > 0, _H3P_KS_WO, _H3P_KS_W2, streams.SIDE_KSPLIT,
           streams.SIDE_KSPLIT_SMALL, _attn_ds(S))
    prog = progs.get(key)
    if prog is None:
        from hetseq_amd.ops.layer_prog import LayerProgram

        rows = B * S
        H, F = W.wo.shape[0], W.w1.shape[0]

        def ksg(M, N):
            return max(streams.side_ksplit(M, N) or 1, -(-rows // 4096))
        prog = LayerProgram(W, Gv, B, S, NH, halves, _H3P_KS_WO, _H3P_KS_W2,
                            {"qkv": ksg(3 * H, H), "wo": ksg(H, H), "w1": ksg(F, H), "w2": ksg(H, F)}, p_a > 0, dev)
        progs[key] = prog
        PROG_BUILDS[0] += 1
    return prog


def _layer_forward_prog(prog, x, mask, W, cfg, am, halves_ok):
    from hetseq_amd.ops import h3p

    B, S, NH, p_h, p_a, eps, seeds = cfg
    (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
    dev = x.device
    xp = h3p.of(x)
    prog.set_input_layout(xp)
    stagger = 0
    if halves_ok:
        fresh = streams.chain_stream() is None  # (the chains' first layer: the fork happens here)
        st1 = streams.chain_fork(dev).cuda_stream
        stagger = _FWD_STAGGER if fresh else 0
    else:
        streams.chain_join(dev)
        st1 = 0
    am0 = G.slot_ptr(am.a(6)) if am is not None else 0
    am1 = G.slot_ptr(am.a(7)) if am is not None and halves_ok else 0
    hip().layer_fwd_h3p(prog.addr, x.data_ptr(), xp.data_ptr(), xp.exps_ptr(), mask.data_ptr(), s_a, o_a, s_1, o_1,
                        s_2, o_2, float(eps), float(p_h), float(p_a), stream_handle(), st1, am0, am1, stagger=stagger)
    streams.chain_keep(x, mask, xp.planes, xp.exps)
    h2 = prog.h2.view(prog.rows, prog.H)
    h3p.remember(h2, prog.h2p)  # the next layer's QKV operand
    return h2, _ProgSaved(prog, xp)


def _layer_backward_prog(ctx, dh2, x, saved, W, meta, cfg):
    B, S, NH, p_h, p_a, eps, seeds = cfg
    (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
    prog, xp = saved.prog, saved.xp
    dh2 = dh2.contiguous()
    dev = dh2.device
    store = meta["store"]
    Gv = meta["grad_sink"]()
    wacc = not (_FRESH_WGRAD and store.claim_fresh())
    for out in (Gv.w2, Gv.w1, Gv.wo, Gv.wqkv):  # lazy zero_grad bookkeeping (runtime/flat.py)
        (store.ensure_zero if wacc else store.mark_stored)(out)
    side = streams.backward_forks(dev, xp.planes, xp.exps)
    if _PROG_SIDE_DELAY:  # (tests: a late side stream -- collectives must still wait for its groups)
        with torch.cuda.stream(side):
            torch.cuda._sleep(_PROG_SIDE_DELAY)
    early = meta.get("early")  # (events address, launch callback): parallel/ddp.py early buckets
    hip().layer_bwd_h3p(prog.addr, dh2.data_ptr(), xp.data_ptr(), xp.exps_ptr(), mask_of(ctx).data_ptr(), s_1, o_1,
                        s_2, o_2, float(p_h), float(p_a), int(wacc), stream_handle(), side.cuda_stream,
                        early[0] if early is not None else 0)
    if early is not None:
        early[1]()
    return (prog.dz1.view(prog.rows, prog.H), None, None) + (None,) * 16


def _layer_forward_h3p(x, mask, W, cfg, save, am=None, meta=None):
    """The layer forward on h3p operands (``W.h3p``: the GEMM weights' planes).  Like
    _layer_forward_split, the batch runs as two half-batch chains on two streams when it splits
    evenly into 128-row halves; each op writes its half of the whole-batch tensors.  Operand planes:
    the layer input's from the previous layer (h3p.recall) or a split pass, the GELU output's from the
    FFN-in GEMM's epilogue (no fp32 copy of it exists), the rest from split passes after their
    producers."""
    from hetseq_amd.ops import h3p

    B, S, NH, p_h, p_a, eps, seeds = cfg
    (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
    Wp = W.h3p
    rows, H = x.shape
    F = W.w1.shape[0]
    dev, f32 = x.device, torch.float32
    halves_ok = (B % 2 == 0 and (rows // 2) % 128 == 0 and rows >= 1024 and streams.enabled() and _FWD_SPLIT)
    prog = _program(W, meta, B, S, NH, p_a, 2 if halves_ok else 1, dev) if (save and meta is not None) else None
    if prog is not None:
        return _layer_forward_prog(prog, x, mask, W, cfg, am, halves_ok)
    if not halves_ok:
        streams.chain_join(dev)
    xp = h3p.of(x)
    qkv = torch.empty((rows, 3 * H), dtype=f32, device=dev)
    ctx_ = torch.empty((rows, H), dtype=f32, device=dev)
    lse = torch.empty((B * NH * S,), dtype=f32, device=dev)
    dmask = torch.empty((B * NH * S * (S // 32),), dtype=torch.int32, device=dev) if p_a > 0 else None
    h1, z1, h2, z2 = (torch.empty((rows, H), dtype=f32, device=dev) for _ in range(4))
    m1, r1, m2, r2 = (torch.empty((rows,), dtype=f32, device=dev) for _ in range(4))
    f1pre = torch.empty((rows, F), dtype=f32, device=dev)
    ctxp, h1p, h2p = (h3p.empty(rows, H, dev) for _ in range(3))
    f1p = h3p.empty(rows, F, dev)
    nh = 2 if halves_ok else 1
    hr, hb = rows // nh, B // nh
    nl, nm = hb * NH * S, hb * NH * S * (S // 32)
    with (streams.fwd_halves(dev) if halves_ok else _OneChain()) as halves:
        for h in halves:
            r = slice(h * hr, (h + 1) * hr)
            r0, r1_ = h * hr, (h + 1) * hr
            sl = (lambda off: am.a(off + h)) if am is not None else (lambda off: None)
            h3p.gemm(xp.rows_slice(r0, r1_), Wp.wqkv, 0, 1, out=qkv[r], site="qkv_fwd")
            attn_fwd_h3p(qkv[r], mask[h * hb:(h + 1) * hb], hb, S, NH, p_a, s_a, o_a, W.bqkv,
                         (ctx_[r], lse[h * nl:(h + 1) * nl], dmask[h * nm:(h + 1) * nm] if dmask is not None else None),
                         h * hb, ctxp.rows_slice(r0, r1_))
            a = h3p.gemm(ctxp.rows_slice(r0, r1_), Wp.wo, 0, 1, ksplit=_H3P_KS_WO, slab_only=True, site="wo_fwd")
            ln_fwd_h3p(a, W.g1, W.b1, eps, W.bo, x[r], p_h, s_1, o_1, (h1[r], z1[r], m1[r], r1[r]), r0,
                       h1p.rows_slice(r0, r1_))
            h3p.gemm(h1p.rows_slice(r0, r1_), Wp.w1, 0, 1, bias=W.bi, epi=h3p.EPI_GELU, aux=f1pre[r],
                     planes_out=f1p.rows_slice(r0, r1_), site="ffn1_fwd")
            o = h3p.gemm(f1p.rows_slice(r0, r1_), Wp.w2, 0, 1, ksplit=_H3P_KS_W2, slab_only=True, site="ffn2_fwd")
            ln_fwd_h3p(o, W.g2, W.bb2, eps, W.b2, h1[r], p_h, s_2, o_2, (h2[r], z2[r], m2[r], r2[r]), r0,
                       h2p.rows_slice(r0, r1_), amax=sl(6))
    h3p.remember(h2, h2p)  # the next layer's QKV operand
    keep = (xp.planes, xp.exps, ctxp.planes, ctxp.exps, h1p.planes, h1p.exps, f1p.planes, f1p.exps, h2p.planes,
            h2p.exps)
    streams.chain_keep(x, mask, qkv, ctx_, lse, dmask, h1, z1, m1, r1, f1pre, h2, z2, m2, r2, *keep)
    if save:
        return h2, (qkv, ctx_, lse, dmask, z1, m1, r1, None, f1pre, None, z2, m2, r2, x, None,
                    ("h3p", xp, ctxp, h1p, f1p))
    return h2, None


def _layer_backward_h3p(ctx, dh2, x, saved, W, meta, cfg):
    """The layer backward on h3p operands: the data-gradient chain on the compute stream, the weight
    gradients on the side stream (split-K slices summed by the reduce pass into the flat store)."""
    from hetseq_amd.ops import h3p

    qkv, ctx_, lse, dmask, z1, m1, r1, _, f1pre, _, z2, m2, r2, _, _, hps = saved
    _, xp, ctxp, h1p, f1p = hps
    Wp = W.h3p
    B, S, NH, p_h, p_a, eps, seeds = cfg
    (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
    dh2 = dh2.contiguous()
    rows, H = dh2.shape
    F = W.w1.shape[0]
    dev = dh2.device
    sink = meta.get("grad_sink")
    Gv = sink() if sink is not None else None
    acc = Gv is not None
    side = acc and streams.enabled()
    store = meta.get("store")
    wacc = acc and not (side and _FRESH_WGRAD and store is not None and store.claim_fresh())
    if not acc:
        Gv = LayerWeights()
        Gv.wqkv = torch.empty_like(W.wqkv)
        Gv.bqkv = torch.zeros(3 * H, dtype=torch.float32, device=dev)
        Gv.wo, Gv.w1, Gv.w2 = torch.empty_like(W.wo), torch.empty_like(W.w1), torch.empty_like(W.w2)
        Gv.bi = torch.zeros(F, dtype=torch.float32, device=dev)

    def wgrad(dyp, xpp, out, site):
        """out (+)= dy^T x on the side stream (or in line without a flat store / side stream)."""
        accumulate = wacc if side else acc
        ks = streams.side_ksplit(out.shape[0], out.shape[1]) if side else 2
        ks = max(ks or 1, -(-rows // 4096))  # a slice is at most 4096 tokens deep

        def run():
            if store is not None:
                (store.ensure_zero if accumulate else store.mark_stored)(out)
            h3p.gemm(dyp, xpp, 1, 0, out=out, beta=1.0 if accumulate else 0.0, ksplit=ks, site=site)
        if side:
            streams.run(dev, run, dyp.planes, dyp.exps, xpp.planes, xpp.exps)
        else:
            run()

    with streams.coalesced():  # LN2 parameter gradients + the FFN-out weight gradient
        da2p = h3p.empty(rows, H, dev)
        dz2, dg2, dbb2, db2 = ln_bwd_h3p(dh2, z2, m2, r2, W.g2, p_h, s_2, o_2, da2p,
                                         acc=(Gv.g2, Gv.bb2, Gv.b2) if acc else None, side=side)
        wgrad(da2p, f1p, Gv.w2, "ffn2_wgrad")
    # FFN-in data gradient through the GELU: planes out only, the FFN-in bias gradient from the
    # epilogue's column partials
    df1p = h3p.empty(rows, F, dev)
    part = torch.empty((rows // 128, F), dtype=torch.float32, device=dev)
    h3p.gemm(da2p, Wp.w2, 0, 0, bias=W.bi, epi=h3p.EPI_DGELU, aux=f1pre, part=part, colsum=Gv.bi,
             colsum_acc=acc, planes_out=df1p, site="ffn2_dgrad")
    wgrad(df1p, h1p, Gv.w1, "ffn1_wgrad")
    h3p.gemm(df1p, Wp.w1, 0, 0, out=dz2, beta=1.0, site="ffn1_dgrad")  # dh1 = dz2 + df1pre @ W1
    with streams.coalesced():  # LN1 parameter gradients + the attention-output weight gradient
        da1p = h3p.empty(rows, H, dev)
        dz1, dg1, db1, dbo = ln_bwd_h3p(dz2, z1, m1, r1, W.g1, p_h, s_1, o_1, da1p,
                                        acc=(Gv.g1, Gv.b1, Gv.bo) if acc else None, side=side)
        wgrad(da1p, ctxp, Gv.wo, "wo_wgrad")
    dctx = h3p.gemm(da1p, Wp.wo, 0, 0, site="wo_dgrad")
    dqkvp = h3p.empty(rows, 3 * H, dev)
    attn_bwd_h3p(qkv, mask_of(ctx), ctx_, dctx, (lse, dmask), B, S, NH, p_a, W.bqkv, dqkvp, fp32=False, ds=_attn_ds(S))
    part_bq = torch.empty(rows // 32, 3 * H, dtype=torch.float32, device=dev)

    def fin_bq():  # the QKV bias gradient: column sums of dqkv's planes (no fp32 dqkv exists)
        h3p_colpart(dqkvp, part_bq)
        hip().colpart_finalize([part_bq.data_ptr()], [Gv.bqkv.data_ptr()], rows // 32, 3 * H, 1, stream_handle())

    with streams.coalesced():  # QKV weight and bias gradients
        wgrad(dqkvp, xp, Gv.wqkv, "qkv_wgrad")
        if side:
            streams.run(dev, fin_bq, part_bq, dqkvp.planes, dqkvp.exps)
        else:
            fin_bq()
    h3p.gemm(dqkvp, Wp.wqkv, 0, 0, out=dz1, beta=1.0, site="qkv_dgrad")  # dx = dz1 + dqkv @ Wqkv
    if acc:
        return (dz1, None, None) + (None,) * 16
    dWqkv, dbqkv = Gv.wqkv, Gv.bqkv
    return (dz1, None, None,
            dWqkv[:H], dbqkv[:H], dWqkv[H:2 * H], dbqkv[H:2 * H], dWqkv[2 * H:], dbqkv[2 * H:],
            Gv.wo, dbo, dg1, db1, Gv.w1, Gv.bi, Gv.w2, db2, dg2, dbb2)


def mask_of(ctx):
    return ctx.saved_tensors[1]


class FusedBertLayer(torch.autograd.Function):
    """One post-LN BERT encoder layer.  Inputs after ``x, mask, meta`` are the
    16 parameters in reference order (q.w, q.b, k.w, k.b, v.w, v.b, o.w, o.b,
    ln1.w, ln1.b, i.w, i.b, out.w, out.b, ln2.w, ln2.b) -- or none, when the layer's
    gradients go straight into a flat store (``meta["grad_sink"]``): autograd then keeps no
    AccumulateGrad node per parameter, and the backward reports the parameters' readiness itself
    (``meta["ready"]``: the data-parallel engine's bucket bookkeeping, parallel/ddp.py)."""

    @staticmethod
    def forward(ctx, x, mask, meta, *params):
        ctx.nparams = len(params)
        W, cfg, recompute = meta["weights"](), meta["cfg"], meta["recompute"]
        # (the native program only for forwards whose backward will run: autograd is off in here)
        h2, saved = _layer_forward(x, mask, W, cfg, save=not recompute, am=meta.get("amax"),
                                   meta=meta if any(ctx.needs_input_grad) else None)
        ctx.meta = meta
        ctx.cfg = cfg
        ctx.h3p = None
        ctx.prog = None
        if isinstance(saved, _ProgSaved):
            ctx.prog = saved
            ctx.save_for_backward(x, mask)
        elif recompute:
            ctx.save_for_backward(x, mask)
        else:
            if len(saved) > 15:  # h3p: the operand planes travel as a ctx attribute (not tensors)
                ctx.h3p = saved[15]
                saved = saved[:15]
            ctx.save_for_backward(x, mask, *saved)
        return h2

    @staticmethod
    def backward(ctx, dh2):
        grads = FusedBertLayer._backward(ctx, dh2)
        if ctx.nparams == 0:
            ready = ctx.meta.get("ready")
            if ready is not None:
                ready()
            return grads[:3]
        return grads

    @staticmethod
    def _backward(ctx, dh2):
        meta, cfg = ctx.meta, ctx.cfg
        W = meta["weights"]()
        if ctx.prog is not None:
            return _layer_backward_prog(ctx, dh2, ctx.saved_tensors[0], ctx.prog, W, meta, cfg)
        if meta["recompute"]:
            x, mask = ctx.saved_tensors
            with torch.no_grad():
                _, saved = _layer_forward(x, mask, W, cfg, save=True, am=meta.get("amax"))
        else:
            x, mask = ctx.saved_tensors[:2]
            saved = ctx.saved_tensors[2:] + (ctx.h3p,)
        if isinstance(saved[-1], tuple) and saved[-1][0] == "h3p":
            return _layer_backward_h3p(ctx, dh2, x, saved, W, meta, cfg)
        qkv, ctx_, lse, dmask, z1, m1, r1, h1, f1pre, f1, z2, m2, r2, xin, cin = saved[:15]
        am = meta.get("amax")  # h3 engine: operand |max| slots (LayerAmax)
        sl = (lambda off, n=1: am.a(off, n)) if am is not None else (lambda off, n=1: None)
        wsl = (lambda i: am.w[i]) if am is not None else (lambda i: None)
        B, S, NH, p_h, p_a, eps, seeds = cfg
        (s_a, o_a), (s_1, o_1), (s_2, o_2) = seeds
        dh2 = dh2.contiguous()
        H = x.shape[1]
        sink = meta.get("grad_sink")
        Gv = sink() if sink is not None else None  # flat-store gradient views (accumulate in place)
        acc = Gv is not None
        # LN2 (bias-dropout-residual) backward
        # weight / bias / LN-parameter gradients go into the flat store on the side stream
        # (runtime/streams.py) and overlap the data-gradient chain; without a flat store they
        # stay in order
        side = acc and streams.enabled()
        dks = streams.DGRAD_KSPLIT if side else None  # K split of the dgrads beside the side stream
        # first backward after zero_grad: the weight gradients are the only writers of their regions
        # and store instead of accumulating (the split-K reduce does not read the zeros back)
        store = meta.get("store")
        wacc = acc and not (side and _FRESH_WGRAD and store is not None and store.claim_fresh())

        def claim(out, accumulate):  # lazy zero_grad bookkeeping (runtime/flat.py): on the writer's stream
            if store is not None and out is not None:
                if accumulate:
                    store.ensure_zero(out)
                else:
                    store.mark_stored(out)

        def wgrad(dy, xin_, out, amax=None):
            if not side:
                claim(out, acc)
                return G.linear_wgrad(dy, xin_, out=out, accumulate=acc, amax=amax)
            ks = streams.side_ksplit(dy.shape[1], xin_.shape[1])

            def run():
                claim(out, wacc)
                return G.linear_wgrad(dy, xin_, out=out, accumulate=wacc, ksplit=ks, amax=amax)
            return streams.run(dy.device, run, dy, xin_)

        def wgrad_bias(dy, xin_, wout, bout, amax):  # side stream: weight + bias gradient, one launch if served
            ks = streams.side_ksplit(dy.shape[1], xin_.shape[1])

            def run_colsum():
                claim(wout, wacc)
                return G.linear_wgrad_colsum(dy, xin_, wout, bout, ksplit=ks, accumulate=wacc, amax=amax)
            if streams.run(dy.device, run_colsum, dy, xin_):
                return wout, bout
            w_ = wgrad(dy, xin_, wout, amax=amax)
            return w_, streams.run(dy.device, lambda: colsum(dy, acc=bout), dy)

        # side-stream work forks at three points per layer; the launches at one point share one event
        with streams.coalesced():  # LN2 parameter gradients + the FFN-out weight gradient
            dz2, do_, dg2, dbb2, db2 = ln_bwd(dh2, z2, m2, r2, W.g2, p_h, 1, s_2, o_2, True, True,
                                              acc=(Gv.g2, Gv.bb2, Gv.b2) if acc else None, side=side, amax=sl(8))
            dW2 = wgrad(do_, f1, Gv.w2 if acc else None, amax=_am(am, sl(8), sl(4, 2)))
        bi_in_wgrad = side and _WGRAD_COLSUM and _FFN_BIAS_WGRAD
        df1p, dbi = G.linear_dgrad_dgelu(do_, W.w2, f1pre, W.bi, db_acc=Gv.bi if acc else None,
                                         amax=_am(am, sl(8), wsl(3)), amax_out=sl(9), colsum=not bi_in_wgrad)
        if dbi is None:  # the bias gradient comes with the FFN-in weight gradient (side stream)
            dW1, dbi = wgrad_bias(df1p, h1, Gv.w1, Gv.bi, _am(am, sl(9), sl(0, 2)))
        else:
            dW1 = wgrad(df1p, h1, Gv.w1 if acc else None, amax=_am(am, sl(9), sl(0, 2)))
        dh1 = G.linear_dgrad(df1p, W.w1, out=dz2, accumulate=True, ksplit=dks,
                             amax=_am(am, sl(9), wsl(2)))  # dz2 + df1pre @ W1
        with streams.coalesced():  # LN1 parameter gradients + the attention-output weight gradient
            dz1, da1, dg1, db1, dbo = ln_bwd(dh1, z1, m1, r1, W.g1, p_h, 1, s_1, o_1, True, True,
                                             acc=(Gv.g1, Gv.b1, Gv.bo) if acc else None, side=side, amax=sl(10))
            dWo = wgrad(da1, cin, Gv.wo if acc else None, amax=_am(am, sl(10), sl(2, 2)))
        dctx = G.linear_dgrad(da1, W.wo, ksplit=dks, amax=_am(am, sl(10), wsl(1)))
        dqkv = attn_bwd(qkv, mask, ctx_, dctx, (lse, dmask), B, S, NH, p_a, bias=W.bqkv, amax=sl(11))
        qkv_w_am = _am(am, sl(11), am and am.xw)
        with streams.coalesced():  # QKV weight and bias gradients
            fused = False
            if side and _WGRAD_COLSUM:  # one launch: the bias gradient from the wgrad's staging
                ks = streams.side_ksplit(dqkv.shape[1], xin.shape[1])

                def run_colsum():
                    claim(Gv.wqkv, wacc)
                    return G.linear_wgrad_colsum(dqkv, xin, Gv.wqkv, Gv.bqkv, ksplit=ks, accumulate=wacc,
                                                 amax=qkv_w_am)
                fused = streams.run(dqkv.device, run_colsum, dqkv, xin)
            if fused:
                dWqkv, dbqkv = Gv.wqkv, Gv.bqkv
            else:
                dWqkv = wgrad(dqkv, xin, Gv.wqkv if acc else None, amax=qkv_w_am)
                if side:
                    dbqkv = streams.run(dqkv.device, lambda: colsum(dqkv, acc=Gv.bqkv), dqkv)
                else:
                    dbqkv = colsum(dqkv, acc=Gv.bqkv if acc else None)
        dx = G.linear_dgrad(dqkv, W.wqkv, out=dz1, accumulate=True, ksplit=dks,
                            amax=_am(am, sl(11), wsl(0)))  # dz1 + dqkv @ Wqkv
        if acc:
            return (dx, None, None) + (None,) * 16
        return (dx, None, None,
                dWqkv[:H], dbqkv[:H], dWqkv[H:2 * H], dbqkv[H:2 * H], dWqkv[2 * H:], dbqkv[2 * H:],
                dWo, dbo, dg1, db1, dW1, dbi, dW2, db2, dg2, dbb2)


# --------------------------------------------------------------------- MLM head + loss
def mlm_compact(labels_flat, cap, ignore_index=-1):
    rows = labels_flat.numel()
    dev = labels_flat.device
    idx = torch.empty(cap, dtype=torch.int32, device=dev)
    lab = torch.empty(cap, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    hip().mlm_compact(labels_flat.data_ptr(), rows, ignore_index, cap, idx.data_ptr(), lab.data_ptr(), cnt.data_ptr(),
                      _err_flag(dev).data_ptr(), stream_handle())
    return idx, lab, cnt


def gather_rows(src, idx):
    n = idx.numel()
    H = src.shape[1]
    out = torch.empty((n, H), dtype=src.dtype, device=src.device)
    hip().gather_rows(dtype_code(src), src.data_ptr(), idx.data_ptr(), out.data_ptr(), n, H, stream_handle())
    return out


def xent_fwd(logits, labels, ignore_index=-1):
    rows, V = logits.shape
    dev = logits.device
    row_loss = torch.empty(rows, dtype=torch.float32, device=dev)
    lse = torch.empty(rows, dtype=torch.float32, device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    hip().xent_fwd(dtype_code(logits), logits.data_ptr(), labels.data_ptr(), rows, V, logits.stride(0), ignore_index,
                   row_loss.data_ptr(), lse.data_ptr(), out.data_ptr(), stream_handle())
    return out, lse


def xent_bwd_(logits, labels, lse, dloss, stats, ignore_index=-1, amax=None):
    """dlogits in place; ``amax``: a zeroed |max| slot the kernel maxes the written values into."""
    rows, V = logits.shape
    hip().xent_bwd(dtype_code(logits), logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), rows, V,
                   logits.stride(0), ignore_index, dloss.data_ptr(), stats.data_ptr(), stream_handle(),
                   amax=G.slot_ptr(amax))
    return logits


class FusedCrossEntropy(torch.autograd.Function):
    """mean CE over rows whose label != ignore_index (reference CrossEntropyLoss(ignore_index=-1))."""

    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        logits = logits.contiguous()
        out, lse = xent_fwd(logits, labels, ignore_index)
        ctx.save_for_backward(logits, labels, lse, out)
        ctx.ignore = ignore_index
        return out[0]

    @staticmethod
    def backward(ctx, dloss):
        logits, labels, lse, out = ctx.saved_tensors
        d = logits.clone()
        xent_bwd_(d, labels, lse, dloss.reshape(1).float().contiguous(), out, ctx.ignore)
        return d, None, None


def _dec_dgrad_ks(K):
    """K slices of the tied decoder's data gradient on planes (K = the padded vocabulary, 30 output
    tiles at BERT-base): slices of <= 2048 (16 at 30720), within the kernel's 4096 per slice."""
    s = 1
    while K // s > 2048 and K % (64 * s) == 0:
        s *= 2
    return s


def cross_entropy(logits, labels, ignore_index=-1):
    return FusedCrossEntropy.apply(logits, labels, ignore_index)


class FusedPreTrainingLoss(torch.autograd.Function):
    """Both pre-training heads and their losses: sparse masked-LM head + CE and pooler + NSP head
    + CE, returning mlm_loss + nsp_loss (reference bert_modeling.py:875-888).

    MLM: exact w.r.t. the dense reference -- rows with label -1 contribute neither loss nor
    gradient, so only the (at most ``cap``) labelled rows go through the transform, the tied
    decoder GEMM and the CE.  Pooler/NSP (K08, pool_nsp.hip): first-token rows read in place,
    fp32 whatever the compute dtype, the final sum done in the NSP loss kernel; its input gradient
    is added straight into the first-token rows of the MLM path's sequence gradient."""

    @staticmethod
    def forward(ctx, seq, labels, nsp_labels, meta, wt, bt, g, b, wdec, bdec, wp, bp, wn, bn):
        T, H = seq.shape
        B, S = meta["B"], meta["S"]
        assert T == B * S and H % 4 == 0 and nsp_labels.dtype == torch.int64 and nsp_labels.numel() == B
        cap, eps = meta["cap"], meta["eps"]
        Wt, Wd = meta["weights"]()
        idx, lab, cnt = mlm_compact(labels.reshape(-1), cap)
        hsel = gather_rows(seq, idx)
        hsel_in = hsel
        hpw = meta.get("h3p")  # h3p engine: (transform planes, tied decoder planes padded to pad512(V) rows)
        ctx.hp = None
        if hpw is not None:
            # every product on block-scaled planes: the gathered rows split once, the transform's GELU
            # in its GEMM epilogue (pre-activation kept), the transform LN writing t2's planes, the
            # decoder over the padded vocabulary (zero weight rows, bias past V read as zero)
            from hetseq_amd.ops import h3p

            Wtp, Wdp = hpw
            R, V = hsel.shape[0], Wd.shape[0]
            hselp = h3p.split(hsel)
            t1pre = torch.empty((R, H), dtype=torch.float32, device=seq.device)
            t1 = h3p.gemm(hselp, Wtp, tb=True, bias=bt, epi=h3p.EPI_GELU, aux=t1pre, site="mlm transform fwd")
            outs = (torch.empty_like(t1), torch.empty_like(t1), torch.empty(R, dtype=torch.float32, device=seq.device),
                    torch.empty(R, dtype=torch.float32, device=seq.device))
            t2p = h3p.empty(R, H, seq.device)
            ln_fwd_h3p(t1, g, b, eps, None, None, 0.0, 0, 0, outs, 0, t2p, region=2)
            t2, z, mean, rstd = outs
            lbuf = torch.empty((R, Wdp.rows), dtype=torch.float32, device=seq.device)
            h3p.gemm(t2p, Wdp, tb=True, out=lbuf, bias=bdec, epi=h3p.EPI_BIAS, valid=(R, V), site="decoder fwd")
            logits = lbuf[:, :V]
            ctx.hp = (hselp, t2p, Wtp, Wdp)
        am = meta.get("amax")  # h3 engine: {seq, wt, wd, t2} |max| slots (hsel's bound: the whole sequence output)
        if hpw is None:
            t1pre = G.linear_fwd(hsel_in, Wt, amax=(am["seq"], am["wt"]) if am else None)
            t1 = bias_gelu_fwd(t1pre, bt)
            t2, z, mean, rstd = ln_fwd(t1, g, b, eps, amax=am["t2"] if am else None)
            # tied decoder on the compacted rows; fp32: the padded split kernel (logits is a view of a
            # zero-padded buffer the backward reuses); bf16: the plane engine
            bfp = meta.get("bf16pad")  # bf16: (the tied decoder's weight padded to pad512(V) rows, bias buffer)
            if t2.dtype == torch.float32:
                logits, lbuf = G.decoder_logits(t2, Wd, bdec, amax=(am["t2"], am["wd"]) if am else None)
            elif bfp is not None:
                # the plane kernels over the padded vocabulary (zero weight rows, zero bias past V): no
                # library GEMM in the bf16 step; logits is a view of the zero-padded buffer
                wdp, bpad = bfp  # (not `bp`: that name is the pooler bias below)
                V = Wd.shape[0]
                bpad[:V].copy_(bdec)
                lbuf = torch.empty((t2.shape[0], wdp.shape[0]), dtype=torch.float32, device=seq.device)
                G.gemm(t2, wdp, tb=True, out=lbuf, bias=bpad, epi=1)
                logits = lbuf[:, :V]
            else:
                logits, lbuf = G.gemm(t2, Wd, tb=True, bias=bdec, epi=1, out_dtype=torch.float32), None
        out, lse = xent_fwd(logits, lab)
        # pooler + NSP + CE; total = out[0] + nsp mean loss
        dev = seq.device
        pooled = torch.empty((B, H), dtype=torch.float32, device=dev)
        nsp_small = torch.empty((B, 4), dtype=torch.float32, device=dev)  # [:, :2] logits, [:, 2] lse
        stats = torch.empty(3, dtype=torch.float32, device=dev)  # count, nsp loss, total
        nsp_logits, nsp_lse = nsp_small[:, :2].contiguous(), nsp_small[:, 2].contiguous()
        hip().pool_nsp_fwd(dtype_code(seq), seq.data_ptr(), B, S, H, wp.data_ptr(), bp.data_ptr(), wn.data_ptr(),
                           bn.data_ptr(), nsp_labels.data_ptr(), out.data_ptr(), pooled.data_ptr(),
                           nsp_logits.data_ptr(), nsp_lse.data_ptr(), stats.data_ptr(), stats[2:].data_ptr(),
                           stream_handle())
        ctx.padded = lbuf is not None
        ctx.bfp = meta.get("bf16pad") if (hpw is None and lbuf is not None and t2.dtype == torch.bfloat16) else None
        ctx.save_for_backward(idx, lab, hsel, t1pre, t1, z, mean, rstd, t2,
                              lbuf if lbuf is not None else logits, lse, out, g, bt, seq, nsp_labels, pooled,
                              nsp_logits, nsp_lse, stats, wp, wn)
        ctx.meta = meta
        ctx.T = T
        return stats[2]

    @staticmethod
    def backward(ctx, dloss):
        (idx, lab, hsel, t1pre, t1, z, mean, rstd, t2, logits, lse, out, g, bt, seq, nsp_labels, pooled, nsp_logits,
         nsp_lse, stats, wp, wn) = ctx.saved_tensors
        meta = ctx.meta
        lbuf = None
        if ctx.padded:  # zero-padded [R, pad512(V)] buffer: the loss works on its [:, :V] view
            lbuf, logits = logits, logits[:, :meta["weights"]()[1].shape[0]]
        Wt, Wd = meta["weights"]()
        sink = meta.get("grad_sink")
        Gv = sink() if sink is not None else None  # (wt, bt, g, b, wdec, bdec, wp, bp, wn, bn) flat-store views
        acc = Gv is not None
        dloss = dloss.reshape(1).float().contiguous()
        am = meta.get("amax")
        # in place, fp32; with the h3 engine it also reports |dlogits| (both decoder gradients' operand)
        dlogits = xent_bwd_(logits, lab, lse, dloss, out, amax=am["dl"] if (am and ctx.padded) else None)
        # tied decoder weight: accumulates into the word-embedding gradient
        # bf16 mode: both decoder GEMMs take bf16 operands (fp32 C for the weight gradient);
        # the fp32-operand weight GEMM cost 268 us vs 72 us (tools/bench_mlm_head.py)
        dl_c = dlogits.to(t2.dtype) if t2.dtype != torch.float32 else dlogits
        bfp = ctx.bfp
        if bfp is not None:  # bf16 padded decoder: the loss gradient over the padded vocabulary (pad columns zero)
            dl_c = lbuf.to(torch.bfloat16)
        # parameter gradients on the weight-gradient stream when they go to the flat store (the
        # decoder one lands in the tied word-embedding gradient: FusedEmbedding.backward waits)
        side = acc and streams.enabled()
        V = dlogits.shape[1]
        # first backward after zero_grad: the decoder GEMM is the first writer of the tied table's
        # gradient (the embedding backward adds its rows later): it stores, the 94 MB of zeros unread
        store = meta.get("store")
        dec_acc = not (side and _FRESH_WGRAD and store is not None and store.claim_fresh())
        am_dl = am["dl"] if (am and lbuf is not None) else None
        hpw = ctx.hp
        if hpw is not None:  # h3p: dlogits split once (pad columns zero); both decoder gradients on planes
            from hetseq_amd.ops import h3p

            hselp, t2p, Wtp, Wdp = hpw
            dlp = h3p.split(lbuf)

            def dwdec():
                if acc and store is not None:
                    (store.ensure_zero if dec_acc else store.mark_stored)(Gv[4])
                out_w = Gv[4] if acc else torch.zeros((V, t2.shape[1]), dtype=torch.float32, device=t2.device)
                return h3p.gemm(dlp, t2p, ta=True, out=out_w, beta=1.0 if dec_acc else 0.0, valid=(V, t2.shape[1]),
                                site="decoder wgrad")
        elif bfp is not None:  # bf16 plane kernels over the padded vocabulary (C rows past V untouched)
            def dwdec():
                if acc and store is not None:
                    (store.ensure_zero if dec_acc else store.mark_stored)(Gv[4])
                out_w = Gv[4] if acc else torch.zeros((V, t2.shape[1]), dtype=torch.float32, device=t2.device)
                return G.decoder_wgrad_bf16(dl_c, t2, V, out_w, accumulate=dec_acc or not acc)
        elif lbuf is not None:  # padded split-bf16 decoder products (pad columns of dlogits stay zero)
            def dwdec():
                if acc and store is not None:  # lazy zero_grad bookkeeping, on the writer's stream
                    (store.ensure_zero if dec_acc else store.mark_stored)(Gv[4])
                out_w = Gv[4] if acc else torch.zeros((V, t2.shape[1]), dtype=torch.float32, device=t2.device)
                return G.decoder_wgrad(lbuf, t2, V, out_w, accumulate=dec_acc,
                                       amax=(am_dl, am["t2"]) if am_dl is not None else None)
        else:
            def dwdec():
                if acc and store is not None:
                    store.ensure_zero(Gv[4])
                return G.linear_wgrad(dl_c, t2, out=Gv[4] if acc else None, accumulate=acc)

        def dbias():
            if lbuf is None:
                return colsum(dlogits, acc=Gv[5] if acc else None)
            full = colsum(lbuf)[:V]  # column sums of the padded buffer (pad columns are zero)
            return Gv[5].add_(full) if acc else full

        if side:
            with streams.coalesced():  # (the mark records on the side stream: one fork serves both)
                dWdec = streams.run(dl_c.device, dwdec, dl_c, t2, lbuf,
                                    *((dlp.planes, dlp.exps, t2p.planes, t2p.exps) if hpw is not None else ()))
                streams.mark(dl_c.device, "tied")  # the embedding backward waits for this GEMM only
                dbdec = streams.run(dl_c.device, dbias, dlogits, lbuf)
        else:
            dWdec = dwdec()
            dbdec = dbias()
        if acc:  # the tied table's dense part is complete: the data-parallel engine reduces it now
            h = tied.lookup(Gv[4])
            if h is not None:
                h.dense_ready(dl_c.device)
        if hpw is not None:  # K = the padded vocabulary over 30 output tiles: 16 K slices
            dt2 = h3p.gemm(dlp, Wdp, ksplit=_dec_dgrad_ks(dlp.cols), site="decoder dgrad")
        elif bfp is not None:  # K = the padded vocabulary (zero rows / columns past V)
            dt2 = G.gemm(dl_c, bfp[0])
        elif lbuf is not None:
            dt2 = G.decoder_dgrad(lbuf, Wd, V, amax=(am_dl, am["wd"]) if am_dl is not None else None)
        else:
            dt2 = G.gemm(dl_c, Wd)
        dt1, _, dg, db, _ = ln_bwd(dt2, z, mean, rstd, g, 0.0, 0, acc=(Gv[2], Gv[3]) if acc else None, side=side)
        am_d = am["dt"] if am else None  # |dt1pre|: the transform's two gradient products share it
        dt1pre, dbt = gelu_bwd_colsum(dt1, t1pre, bt, db_acc=Gv[1] if acc else None, amax=am_d)
        hsel_in, dt1pre_in = hsel, dt1pre
        if hpw is not None:  # the transform's gradients on planes (dt1pre split once)
            dtp = h3p.split(dt1pre)

            def dwt():
                out_t = Gv[0] if acc else torch.zeros_like(Wt)
                return h3p.gemm(dtp, hselp, ta=True, out=out_t, beta=1.0, site="mlm transform wgrad")
            dWt = streams.run(dt1pre.device, dwt, dtp.planes, dtp.exps, hselp.planes, hselp.exps) if side else dwt()
            dhsel = h3p.gemm(dtp, Wtp, site="mlm transform dgrad")
        else:
            wt_am = (am_d, am["seq"]) if am else None
            if side:
                dWt = streams.run(dt1pre.device, lambda: G.linear_wgrad(dt1pre_in, hsel_in, out=Gv[0], accumulate=True,
                                                                        amax=wt_am), dt1pre_in, hsel_in, am_d)
            else:
                dWt = G.linear_wgrad(dt1pre_in, hsel_in, out=Gv[0] if acc else None, accumulate=acc, amax=wt_am)
            dhsel = G.linear_dgrad(dt1pre_in, Wt, amax=(am_d, am["wt"]) if am else None)
        H_ = seq.shape[1]
        dseq = torch.zeros((ctx.T, H_), dtype=seq.dtype, device=seq.device)
        hip().scatter_add_rows(dtype_code(dseq), dhsel.data_ptr(), idx.data_ptr(), dseq.data_ptr(), idx.numel(),
                               H_, stream_handle())
        # pooler / NSP: input gradient added into dseq's first-token rows; parameter gradients
        # written (or accumulated into the flat store) by the deterministic column kernel
        B, S, H = meta["B"], meta["S"], seq.shape[1]
        dev = seq.device
        if acc:
            dWp, dbp, dWn, dbn = Gv[6], Gv[7], Gv[8], Gv[9]
        else:
            dWp = torch.empty((H, H), dtype=torch.float32, device=dev)
            dbp = torch.empty(H, dtype=torch.float32, device=dev)
            dWn = torch.empty((2, H), dtype=torch.float32, device=dev)
            dbn = torch.empty(2, dtype=torch.float32, device=dev)
        scratch = torch.empty(B * (2 + 9 * H), dtype=torch.float32, device=dev)  # dlogits, dpre, 8 dx chunks
        dnsp, dpre, part = scratch[:2 * B], scratch[2 * B:2 * B + B * H], scratch[2 * B + B * H:]
        hip().pool_nsp_bwd(dtype_code(seq), dloss.data_ptr(), seq.data_ptr(), dseq.data_ptr(), B, S, H,
                           wp.data_ptr(), wn.data_ptr(), nsp_labels.data_ptr(), pooled.data_ptr(),
                           nsp_logits.data_ptr(), nsp_lse.data_ptr(), stats.data_ptr(), dnsp.data_ptr(),
                           dpre.data_ptr(), part.data_ptr(), dWp.data_ptr(), dbp.data_ptr(), dWn.data_ptr(),
                           dbn.data_ptr(), int(acc), stream_handle(), with_wgrad=0)

        def pool_wgrad():  # the pooler / NSP parameter gradients: off the data-gradient chain
            hip().pool_nsp_wgrad(dtype_code(seq), seq.data_ptr(), dpre.data_ptr(), dnsp.data_ptr(), pooled.data_ptr(),
                                 B, S, H, dWp.data_ptr(), dbp.data_ptr(), dWn.data_ptr(), dbn.data_ptr(), int(acc),
                                 stream_handle())
        if side and _POOL_WGRAD_SIDE:
            streams.run(dev, pool_wgrad, seq, scratch, pooled, dWp, dbp, dWn, dbn)
        else:
            pool_wgrad()
        if acc:
            return (dseq,) + (None,) * 13
        return (dseq, None, None, None, dWt, dbt, dg, db, dWdec, dbdec, dWp, dbp, dWn, dbn)
