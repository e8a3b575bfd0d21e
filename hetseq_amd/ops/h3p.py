"""Block-scaled split-fp16 operands ("h3p") and the GEMM over them (csrc/kernels/gemm_h3p.hip).

An fp32 matrix ``X [R, C]`` (R, C multiples of 32) is held as :class:`HP`: two fp16 planes
(hi, lo) and one int8 exponent per 32 x 32 block, ``x * 2^e = hi + lo`` to 2^-22 (format:
csrc/kernels/h3p.h).  Producing kernels write this format next to (or instead of) their fp32
output -- the LayerNorm forward / backward, the attention kernels, the FFN GEMM's GELU / dGELU
epilogues -- and :func:`split` does it for any other fp32 matrix (the weights, once per update).
The GEMM then runs three fp16 MFMA products per fp32 product with no split work in its K loop.

Precision: every element keeps 22 significant bits inside a 2^18 window below its OWN 32 x 32
block's largest magnitude (the previous engine, gemm.hip NT=4, had one window per tensor), the
products are exact in the fp32 accumulator, and block factors are applied once per 32-deep K tile
to an accumulator that holds true fp32 values (tests/test_h3p_gpu.py measures it against fp64 next
to exact-fp32 products).  Reference: the fp32 Linears of bert_modeling.py:352-354, 166-172,
423-427 and their autograd backward.
"""
from __future__ import annotations

import struct
import weakref

import torch

from hetseq_amd.ops._C import hip, stream_handle

BLK = 32
EPI_NONE, EPI_BIAS, EPI_GELU, EPI_DGELU = 0, 1, 2, 3


class HP(object):
    """h3p planes of an fp32 ``[rows, cols]`` matrix: ``planes`` [2, rows, ld] fp16 (hi, lo) and
    ``exps`` [rows/32, cols/32] int8.  ``rows`` may be a row window of a larger allocation
    (:meth:`rows_slice`: ``offset`` elements into ``planes``, ``eoff`` into ``exps``).  ``blk``: the
    planes' layout -- True blocked (32 x 32 blocks of 2 KB per plane: h3p.h; what every producer
    kernel writes), False row-major (the split pass and the GEMM read both; tests)."""

    __slots__ = ("planes", "exps", "rows", "cols", "ld", "ps", "offset", "eoff", "lde", "blk")

    def __init__(self, planes, exps, rows, cols, ld=None, ps=None, offset=0, eoff=0, lde=None, blk=True):
        self.planes, self.exps = planes, exps
        self.rows, self.cols = rows, cols
        self.ld = cols if ld is None else ld
        self.ps = planes[0].numel() if ps is None else ps
        self.offset, self.eoff = offset, eoff
        self.lde = cols // BLK if lde is None else lde
        self.blk = bool(blk)

    @property
    def shape(self):
        return (self.rows, self.cols)

    @property
    def device(self):
        return self.planes.device

    @property
    def is_cuda(self):
        return self.planes.is_cuda

    def data_ptr(self):
        return self.planes.data_ptr() + 2 * self.offset

    def exps_ptr(self):
        return self.exps.data_ptr() + self.eoff

    def rows_slice(self, r0, r1):
        """The planes of rows [r0, r1) (multiples of 32): a view, no copy."""
        assert r0 % BLK == 0 and r1 % BLK == 0 and 0 <= r0 < r1 <= self.rows
        return HP(self.planes, self.exps, r1 - r0, self.cols, self.ld, self.ps, self.offset + r0 * self.ld,
                  self.eoff + (r0 // BLK) * self.lde, self.lde, self.blk)

    def plane(self, p):
        """Plane ``p`` (0 hi, 1 lo) as an fp16 ``[rows, cols]`` tensor (a copy when blocked)."""
        flat = self.planes.reshape(-1).view(torch.float16)
        off = self.offset + p * self.ps
        if not self.blk:
            return torch.as_strided(flat, (self.rows, self.cols), (self.ld, 1), off)
        v = torch.as_strided(flat, (self.rows // BLK, self.cols // BLK, BLK, BLK), (BLK * self.ld, BLK * BLK, BLK, 1),
                             off)
        return v.permute(0, 2, 1, 3).reshape(self.rows, self.cols)

    def unsplit(self):
        """fp32 value (hi + lo) * 2^-e (tests / diagnostics)."""
        hi, lo = self.plane(0).float(), self.plane(1).float()
        e = torch.as_strided(self.exps.reshape(-1), (self.rows // BLK, self.cols // BLK), (self.lde, 1),
                             self.eoff).to(torch.float32)
        scale = torch.exp2(-e).repeat_interleave(BLK, 0).repeat_interleave(BLK, 1)
        return (hi.double() + lo.double()).float() * scale


def empty(rows, cols, device, blk=True):
    """Uninitialised HP storage for a producer kernel to fill."""
    assert rows % BLK == 0 and cols % BLK == 0
    planes = torch.empty((2, rows, cols), dtype=torch.int16, device=device)
    exps = torch.empty((rows // BLK, cols // BLK), dtype=torch.int8, device=device)
    return HP(planes, exps, rows, cols, blk=blk)


def split(x, out=None, blk=True, rows=None):
    """fp32 ``[rows, cols]`` (row-major, cols a multiple of 32) -> :class:`HP` (one pass: one wave per
    32 x 32 block); ``blk``: blocked plane layout (ignored when ``out`` is given).  ``rows`` (a multiple
    of 32, >= x's rows): the planes' row count -- x's missing rows split as zeros (a padded vocabulary)."""
    assert x.dtype == torch.float32 and x.dim() == 2 and x.stride(1) == 1
    vrows, cols = x.shape
    rows = out.rows if out is not None else (vrows if rows is None else rows)
    hp = out if out is not None else empty(rows, cols, x.device, blk)
    hip().h3p_split(x.data_ptr(), x.stride(0), rows, cols, hp.data_ptr(), hp.ld, hp.ps, hp.exps_ptr(), hp.lde,
                    stream_handle(), int(hp.blk), vrows)
    return hp


class SplitTable(object):
    """One launch that splits many fp32 matrices (the GEMM weights after every update): the
    segment records live in device memory, built once for fixed addresses."""

    FMT = "QQQqqqqiiiiii"  # QSplitSeg (gemm_h3p.hip): src, dst, ex, lds, ldd, ps, lde, rows, cols, blk0, blocked, vrows, pad

    def __init__(self, pairs, device):
        """``pairs``: [(fp32 2-D tensor, HP destination)]; a tensor with fewer rows than its destination
        (a vocabulary padded to the GEMM tile) splits the missing rows as zeros."""
        nbytes = hip().h3p_split_seg_bytes()
        assert struct.calcsize("<" + self.FMT) == nbytes, "QSplitSeg layout changed"
        recs, blk = [], 0
        for x, hp in pairs:
            assert x.dtype == torch.float32 and x.stride(1) == 1 and x.shape[1] == hp.cols and x.shape[0] <= hp.rows
            assert x.data_ptr() % 16 == 0 and x.stride(0) % 4 == 0
            recs.append(struct.pack("<" + self.FMT, x.data_ptr(), hp.data_ptr(), hp.exps_ptr(), x.stride(0), hp.ld,
                                    hp.ps, hp.lde, hp.rows, hp.cols, blk, int(hp.blk), x.shape[0], 0))
            blk += (hp.rows // BLK) * (hp.cols // BLK)
        raw = torch.frombuffer(bytearray(b"".join(recs)), dtype=torch.uint8)
        self.table = raw.to(device)
        self.nseg, self.total = len(recs), blk
        self.keep = pairs  # the addresses in the table stay valid while this object lives

    def run(self, stream=None):
        hip().h3p_split_multi(self.table.data_ptr(), self.nseg, self.total,
                              stream if stream is not None else stream_handle())


_SLABS: dict = {}


def _slab(n, device):
    from hetseq_amd.runtime import streams

    key = (device, streams.role(stream_handle()))
    buf = _SLABS.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(n, dtype=torch.float32, device=device)
        _SLABS[key] = buf
    return buf


def dims(a, b, ta, tb):
    M = a.cols if ta else a.rows
    K = a.rows if ta else a.cols
    N = b.rows if tb else b.cols
    return M, N, K


def ksplit_for(M, N, K):
    """K slices so the grid covers the 256 CUs' two resident blocks (each slice >= 512 deep)."""
    tiles, s = (M // 128) * (N // 128), 1
    while tiles * s < 384 and K % (2 * s * 32) == 0 and K // (2 * s) >= 512 and s < 8:
        s *= 2
    return s


# ------------------------------------------------------------------ precision census
# HETSEQ_H3P_CENSUS=1 (or census_start()): every gemm() records, per call site and operand, how many
# nonzero elements lie below their block's 2^18 window (|x * 2^e| < 2^-3: fewer than 22 bits kept)
# and their share of the operand's |x| mass.  Host-synchronising; a diagnostic (tools/h3p_census.py).
CENSUS: dict = {}
_CENSUS_ON = [__import__("os").environ.get("HETSEQ_H3P_CENSUS", "0") == "1"]


def census_start():
    CENSUS.clear()
    _CENSUS_ON[0] = True


def census_stop():
    _CENSUS_ON[0] = False
    return dict(CENSUS)


def window_stats(hp):
    """(nonzero elements, of them below the window, |x| mass below the window, total |x| mass)."""
    hi = hp.plane(0).float()
    x = hp.unsplit().double()
    nz = x != 0
    out = nz & (hi.abs() < 0.125)
    ax = x.abs()
    return int(nz.sum()), int(out.sum()), float(ax[out].sum()), float(ax.sum())


def window_stats_tensor(hp):
    """window_stats of the SAME values under ONE exponent for the whole tensor (the per-tensor scale of
    the h3 engine): the per-block window can only keep more bits (each block's exponent is >= the
    tensor's), so its counts must be <= these on every tensor -- the census checks it."""
    import math

    x = hp.unsplit().double()
    ax = x.abs()
    m = float(ax.max()) if x.numel() else 0.0
    nz = x != 0
    if not m > 0.0:
        return int(nz.sum()), 0, 0.0, float(ax.sum())
    e = 14 - math.floor(math.log2(m))
    out = nz & (ax * 2.0 ** e < 0.125)
    return int(nz.sum()), int(out.sum()), float(ax[out].sum()), float(ax.sum())


def _census(site, a, b):
    for role, hp in (("A", a), ("B", b)):
        for kind, st in (("", window_stats(hp)), ("/tensor", window_stats_tensor(hp))):
            c = CENSUS.setdefault((site, role + kind), [0, 0, 0.0, 0.0, 0])
            for i in range(4):
                c[i] += st[i]
            c[4] += 1


def gemm(a, b, ta=False, tb=False, out=None, bias=None, epi=EPI_NONE, beta=0.0, aux=None, part=None, colsum=None,
         colsum_acc=False, ksplit=1, planes_out=None, slab_only=False, site=None, valid=None):
    """``out = beta*out + op(a) @ op(b)`` (+ epilogue) on h3p operands.

    ``epi``: EPI_BIAS (+bias), EPI_GELU (``aux`` <- pre-activation, result gelu(pre + bias)),
    EPI_DGELU (result = acc * gelu'(aux + bias), column sums into ``colsum`` via ``part``
    [M/128, N] scratch).  ``planes_out``: an :class:`HP` [M, N] that receives the GELU / dGELU result
    (``out`` may then be None).  ``ksplit`` > 1: fp32 slabs summed by a reduce pass into ``out``, or
    -- ``slab_only`` -- returned as a [ks, M, N] view for a consumer that sums them (valid until
    the next split GEMM on this stream).  ``valid`` = (Mv, Nv): a padded problem's real extents --
    ``out`` ([Mv, N] or [M, N]) gets rows < Mv only, bias entries past Nv read as zero.  Raises on a
    request the kernel does not serve."""
    M, N, K = dims(a, b, ta, tb)
    assert (tb and b.cols == K) or (not tb and b.rows == K), "inner dimensions differ"
    if _CENSUS_ON[0]:
        _census(site or (M, N, K, ta, tb), a, b)
    dev = a.device
    slab = None
    if ksplit > 1:
        slab = _slab(ksplit * M * N, dev)
    elif slab_only:  # one slice: the slab's first plane is C
        out = _slab(M * N, dev)[:M * N].view(M, N)
    if out is None and not slab_only and planes_out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=dev)
    mv, nv = valid if valid is not None else (0, 0)
    if out is not None:
        assert out.dtype == torch.float32 and out.shape[1] == N and out.shape[0] in (M, mv) and out.stride(1) == 1
    assert planes_out is None or planes_out.blk, "the GEMM epilogue writes blocked planes"
    rc = hip().gemm_h3p(int(ta), int(tb), M, N, K, a.data_ptr(), a.ld, a.ps, a.exps_ptr(), a.lde,
                        b.data_ptr(), b.ld, b.ps, b.exps_ptr(), b.lde,
                        out.data_ptr() if out is not None else 0, out.stride(0) if out is not None else N,
                        bias.data_ptr() if bias is not None else 0, int(epi), float(beta),
                        aux.data_ptr() if aux is not None else 0, aux.stride(0) if aux is not None else 0,
                        part.data_ptr() if part is not None else 0, colsum.data_ptr() if colsum is not None else 0,
                        int(colsum_acc),
                        planes_out.data_ptr() if planes_out is not None else 0,
                        planes_out.ld if planes_out is not None else 0, planes_out.ps if planes_out is not None else 0,
                        planes_out.exps_ptr() if planes_out is not None else 0,
                        planes_out.lde if planes_out is not None else 0,
                        int(ksplit), slab.data_ptr() if slab is not None else 0,
                        slab.numel() if slab is not None else 0, stream_handle(), int(a.blk), int(b.blk), int(mv), int(nv))
    if rc != 0:
        raise ValueError("gemm_h3p: request not served (M=%d N=%d K=%d ta=%d tb=%d epi=%d ksplit=%d)"
                         % (M, N, K, ta, tb, epi, ksplit))
    if slab_only:
        return slab[:ksplit * M * N].view(ksplit, M, N) if ksplit > 1 else out.view(1, M, N)
    return out


# HP operands a producer kernel already wrote for an fp32 tensor (the layer output's planes, read by
# the next layer): keyed by the tensor object and its version counter, so an in-place update drops
# the entry; consumed once.
_KNOWN: dict = {}


def remember(t, hp):
    _KNOWN[id(t)] = (weakref.ref(t), t._version, hp)
    if len(_KNOWN) > 16:  # entries of tensors that were never consumed (the last layer's output)
        for k in [k for k, v in _KNOWN.items() if v[0]() is None]:
            del _KNOWN[k]


def recall(t):
    """The HP a producer remembered for ``t`` (None: not known, or ``t`` changed since)."""
    e = _KNOWN.pop(id(t), None)
    if e is not None and e[0]() is t and e[1] == t._version:
        return e[2]
    return None


def of(t):
    """``t``'s HP: the producer's (:func:`recall`) or one split pass."""
    hp = recall(t)
    return hp if hp is not None else split(t.contiguous())


def ok_shape(rows, *cols):
    """Whether the h3p GEMMs tile a layer with ``rows`` tokens and these feature widths."""
    return rows % 128 == 0 and all(c % 128 == 0 for c in cols)
