"""GEMM dispatch for the BERT hot path.

``linear_fwd`` / ``linear_dgrad`` / ``linear_wgrad`` are the three products
of a Linear layer; ``linear_gelu_fwd`` and ``linear_dgrad_dgelu`` are the FFN
products with the GELU (and its backward + bias gradient) fused into the GEMM
epilogue.  Two engines:

* ``hip``  -- the hand-written gfx950 MFMA kernels (csrc/kernels/gemm.hip, gemm_planes.hip,
             gemm_h3p.hip) with fused epilogues (bias, bias+GELU, dGELU+bias-grad,
             beta-accumulate).  The only engine of the training step.
* ``blas`` -- hipBLASLt / rocBLAS through ``torch.mm``: a reference ORACLE for tests and
             benchmarks (``HETSEQ_GEMM=blas`` / :func:`set_mode`), and the fallback for a shape
             no hand-written kernel serves (odd test shapes; never a BERT-base site).

fp32 products on the HIP engine run on the 16-bit matrix cores: as three split-fp16
products with per-tensor power-of-two operand scales (``HETSEQ_FP32_GEMM=h3``: fp32-level
error at half the MFMA work of x6, see gemm.hip ``split4h``; every operand needs its |max|,
which the producing kernels emit -- :func:`amax_of` computes it for the rest), as six split-bf16
products (``x6``: fp32-level error at any dynamic range, no scale needed), or on the exact-fp32 MFMA
(``native``: the accuracy oracle).

``HETSEQ_GEMM=hip|blas`` selects (default ``hip``).  There is no run-time choice between the
hand-written kernels and the library (round 6): per call site only the hand-written kernels'
own variants are measured once (split-K, plane-engine variant), recorded in ``GEMM_CHOICES``
and logged by the benchmark.  In bf16 mode the
weight-gradient GEMM writes fp32 directly (``out_dtype``), so master gradients
never round through bf16.
"""
from __future__ import annotations

import os

import torch

from hetseq_amd.ops._C import hip, stream_handle

GEMM_CHOICES: dict = {}
_MODE = os.environ.get("HETSEQ_GEMM", "hip")
assert _MODE in ("hip", "blas"), "HETSEQ_GEMM must be hip or blas"
# h3p: the encoder layers' products on pre-split block-scaled planes (ops/h3p.py, gemm_h3p.hip); every
# other fp32 product (the pre-training heads, standalone calls) on the h3 engine (dtype code 4)
_FP32_DT = {"native": 0, "x6": 2, "h3": 4, "h3p": 4}
_FP32 = os.environ.get("HETSEQ_FP32_GEMM", "h3p")
FP32_DEFAULT = _FP32
assert _FP32 in _FP32_DT, "HETSEQ_FP32_GEMM must be one of native|x6|h3|h3p"
SPLIT_ENGINES = ("x6", "h3", "h3p")  # the fp32-level split engines
_SLABS: dict = {}  # (device, stream) -> split-K partial-sum workspace

EPI_NONE, EPI_BIAS, EPI_GELU, EPI_DGELU = 0, 1, 2, 3


def gemm_mode():
    """'hip' (the hand-written kernels) or 'blas' (the library oracle)."""
    return _MODE


def set_mode(mode):
    global _MODE
    assert mode in ("hip", "blas")
    _MODE = mode
    GEMM_CHOICES.clear()


def save_choices(path):
    """Write the measured per-call-site engine choices (JSON) so a later run can skip the measuring."""
    import json

    with open(path, "w") as f:
        json.dump({"fp32": _FP32, "choices": {repr(k): v for k, v in GEMM_CHOICES.items()}}, f, indent=0)


def load_choices(path):
    """Load choices written by save_choices (only when they were measured under the same fp32 policy)."""
    import ast
    import json

    with open(path) as f:
        d = json.load(f)
    if d.get("fp32") != _FP32:
        return False
    for k, v in d["choices"].items():
        if v and v[0] == "hip":  # (older files also hold library choices: those sites are re-measured)
            GEMM_CHOICES[ast.literal_eval(k)] = tuple(v)
    return True


# A |max| slot: AMAX_SHARDS partial maxima 64 B apart (csrc/kernels/common.h kAmaxShards): writers
# spread their atomics over the shards, readers max over them
AMAX_SHARDS, AMAX_STRIDE = 32, 16
SLOT_FLOATS = AMAX_SHARDS * AMAX_STRIDE


def amax_value(slot_tensor):
    """The |max| a slot tensor (amax_of's result) holds (tests / diagnostics)."""
    v = slot_tensor.view(-1, AMAX_STRIDE)[:, 0]
    return v.view(-1, AMAX_SHARDS).max(dim=1).values


def amax_of(x, out=None):
    """|max| of fp32 ``x`` as a one-slot device tensor (``out`` if given): the operand scale source of
    the h3 engine for tensors no fused producer reported.  NaN propagates (a NaN |max| leaves the
    operand unscaled, so the NaN reaches the product)."""
    if out is None:
        out = torch.empty(SLOT_FLOATS, dtype=torch.float32, device=x.device)
    if (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.numel() % 4 == 0
            and x.data_ptr() % 16 == 0):
        hip().amax(x.data_ptr(), x.numel(), out.data_ptr(), 1, stream_handle())
    else:
        out.zero_()
        amax_into(x, out)
    return out


def slot_ptr(a):
    """Device address of a |max| slot: a (pointer, count) tuple (AmaxPool slots -- plain ints, no
    tensor view per use), a 1-D fp32 tensor, or None (0)."""
    if a is None:
        return 0
    return a[0] if isinstance(a, tuple) else a.data_ptr()


def amax_into(x, slot):
    """Atomically max |x| into an existing slot (tensor or (pointer, count)) on the current stream."""
    if (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.numel() % 4 == 0
            and x.data_ptr() % 16 == 0):
        hip().amax(x.data_ptr(), x.numel(), slot_ptr(slot), 0, stream_handle())
    else:
        tmp = torch.zeros(4, dtype=torch.float32, device=x.device)
        tmp[0] = x.detach().abs().amax().float() if x.numel() else 0.0
        hip().amax(tmp.data_ptr(), 4, slot_ptr(slot), 0, stream_handle())


def _amax_ptr(t, given, keep):
    """(pointer, count) of an operand's |max| partials for the h3 engine.  A |max| computed here is
    appended to ``keep``: the caller holds it until the GEMM is launched -- freed earlier, the
    caching allocator hands the same 4 bytes to the OTHER operand's |max| and both read one value."""
    if isinstance(given, tuple):
        return given
    am = given if given is not None else amax_of(t)
    assert am.dtype == torch.float32 and am.is_contiguous() and am.numel() % SLOT_FLOATS == 0
    keep.append(am)
    return am.data_ptr(), am.numel() // SLOT_FLOATS


def _h3_census(site, a, b):
    """Precision census of the per-tensor-scaled h3 engine (ops/h3p.py CENSUS, same metric): nonzero
    elements below their TENSOR's 2^18 window (|x * 2^e| < 2^-3, e from the tensor's |max|)."""
    from hetseq_amd.ops import h3p

    if not h3p._CENSUS_ON[0]:
        return
    for role, t in (("A", a), ("B", b)):
        x = t.detach().double()
        ax = x.abs()
        m = float(ax.max()) if x.numel() else 0.0
        if not m > 0.0:
            continue
        import math

        e = 14 - math.floor(math.log2(m))
        nz = x != 0
        out = nz & (ax * 2.0 ** e < 0.125)
        c = h3p.CENSUS.setdefault(("h3",) + tuple(site) + (role,), [0, 0, 0.0, 0.0, 0])
        c[0] += int(nz.sum())
        c[1] += int(out.sum())
        c[2] += float(ax[out].sum())
        c[3] += float(ax.sum())
        c[4] += 1


def set_fp32_mode(mode):
    """'h3p' (encoder layers on block-scaled planes, h3 elsewhere), 'h3' (split-fp16 products,
    per-tensor scales), 'x6' (split-bf16 products, no scale: wide-range data; both fp32-level error)
    or 'native' (exact-fp32 MFMA)."""
    global _FP32
    assert mode in _FP32_DT
    _FP32 = mode
    GEMM_CHOICES.clear()


def fp32_mode():
    return _FP32


def _slab(M, N, ksplit, device):
    """Split-K workspace for ksplit partial [M,N] fp32 planes (grown on demand).  One per stream
    role -- the compute stream (or the graph-capture stream standing in for it) and the
    weight-gradient side stream -- since those two run GEMMs concurrently."""
    from hetseq_amd.runtime import streams

    key = (device, streams.role(stream_handle()))
    need = 8 * M * N if ksplit <= 0 else ksplit * M * N
    buf = _SLABS.get(key)
    if buf is None or buf.numel() < need:
        if torch.cuda.is_current_stream_capturing():
            return None  # never allocate inside a graph capture: run without split-K
        buf = torch.empty(need, dtype=torch.float32, device=device)
        _SLABS[key] = buf
    return buf


# ------------------------------------------------------------------ bf16-plane operands
class Planes(object):
    """A [rows, cols] bf16 GEMM operand of the bf16-plane engine (csrc/kernels/gemm_planes.hip,
    --dtype bf16; P = 1).  ``buf`` owns the storage; element (r, c) sits at flat index
    ``offset + r * ld + c`` of it."""

    __slots__ = ("buf", "rows", "cols", "ld", "ps", "P", "offset")

    def __init__(self, buf, rows, cols, ld, ps, P, offset=0):
        self.buf, self.rows, self.cols, self.ld, self.ps, self.P, self.offset = buf, rows, cols, ld, ps, P, offset

    @property
    def shape(self):
        return (self.rows, self.cols)

    @property
    def device(self):
        return self.buf.device

    @property
    def is_cuda(self):
        return self.buf.is_cuda

    def data_ptr(self):
        return self.buf.data_ptr() + 2 * self.offset

    @staticmethod
    def of_bf16(x):
        """P = 1 view of a row-major bf16 matrix (rows may be strided)."""
        assert x.dtype == torch.bfloat16 and x.dim() == 2 and x.stride(1) == 1
        return Planes(x, x.shape[0], x.shape[1], x.stride(0), 0, 1)

    def unsplit(self):
        """fp32 value (tests / debugging)."""
        v = self.buf.reshape(-1)[self.offset:]
        return torch.as_strided(v, (self.rows, self.cols), (self.ld, 1)).float()


def _unplane(x):
    """The bf16 matrix behind a Planes operand (shapes the plane engine does not tile); other operands
    unchanged."""
    return x.buf if isinstance(x, Planes) else x


def _as_planes(x):
    if isinstance(x, Planes):
        return x
    if x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and x.stride(1) == 1:
        return Planes.of_bf16(x)
    return None


def gemm_planes(a, b, ta, tb, out, bias=None, epi=EPI_NONE, beta=0.0, aux=None, part=None, colsum=None,
                colsum_acc=False, ksplit=1, variant=-1, mv=0):
    """Launch the bf16-plane engine on Planes operands; False (nothing launched) if not served.
    ``variant``: kernel variant (gemm_planes.hip: 0 two LDS stages, 1 one stage, 2 half K depth,
    3 eight waves, 4 eight waves + one stage); -1 = :func:`planes_variant`.  ``mv`` > 0: the valid
    rows of a padded problem (fp32 ``out`` of ``mv`` rows, plain / bias epilogue)."""
    M, N, K = _dims(a, b, ta, tb)
    if out is None or a.P != b.P or not out.is_cuda or out.stride(1) != 1 or \
            out.dtype not in (torch.float32, torch.bfloat16) or out.shape != ((mv or M), N):
        return False
    slab = _slab(M, N, ksplit, out.device) if ksplit > 1 else None
    if ksplit > 1 and slab is None:
        ksplit = 1
    if variant < 0:
        variant = planes_variant(M, N, K, a.P, ta)
    rc = hip().gemm_planes(a.P, 1 if out.dtype == torch.bfloat16 else 0, int(ta), int(tb), M, N, K, a.data_ptr(),
                           a.ld, a.ps, b.data_ptr(), b.ld, b.ps, out.data_ptr(), out.stride(0),
                           bias.data_ptr() if bias is not None else 0, epi, float(beta),
                           aux.data_ptr() if aux is not None else 0, aux.stride(0) if aux is not None else 0,
                           part.data_ptr() if part is not None else 0, colsum.data_ptr() if colsum is not None else 0,
                           int(colsum_acc), int(ksplit), slab.data_ptr() if slab is not None else 0,
                           slab.numel() if slab is not None else 0, int(variant), stream_handle(), mv=int(mv))
    return rc == 0


def planes_variant(M, N, K, P, ta):
    """Default kernel variant per shape (profiles/r2_gemm_engines.md): one LDS stage (3 workgroups per
    CU), except the small-grid 768 x 768-class products (8 waves); call sites are measured (gemm())."""
    tiles = (M // 128) * (N // 128)
    if tiles <= 256 and K <= 1024 and not ta:
        return 3
    return 1


# split-K of the plane engine's weight gradients (K = tokens): slices so the tile grid covers the
# chip about twice; measured choices can override per shape (PLANES_KSPLIT)
PLANES_KSPLIT: dict = {}


def _planes_ksplit(M, N, K, P):
    key = (M, N, K, P)
    if key in PLANES_KSPLIT:
        return PLANES_KSPLIT[key]
    tiles, s = (M // 128) * (N // 128), 1
    while tiles * s < 384 and s < 8 and K % (2 * s * 64) == 0 and K // (2 * s) >= 512:
        s *= 2
    return s


def _bf16_choice(key, pa, pb, ta, tb, out, bias, epi, beta, ks, out_dtype):
    """bf16 operands on the plane engine: its fastest variant and K split for the call site, measured
    once (GEMM_CHOICES).  Returns ``out`` when the engine ran, None for a shape it does not serve."""
    c = GEMM_CHOICES.get(key)
    if c is None and not torch.cuda.is_current_stream_capturing():
        scratch = out.clone() if beta != 0.0 else torch.empty_like(out)
        M, N, K = _dims(pa, pb, ta, tb)
        splits = [ks]
        if not ta and epi in (EPI_NONE, EPI_BIAS) and (M // 128) * (N // 128) < 384:
            # a grid under 1.5 blocks per CU (the N = 768 products): also try K slices (up to 16 for a
            # long K: the tied decoder's data gradient, K = the padded vocabulary over ~30 tiles)
            splits = [s for s in ((1, 2, 4, 8, 16) if K >= 8192 else (1, 2, 4)) if K % (64 * s) == 0]
        best = None
        for s in splits:
            for v in (0, 1, 3, 4):
                if gemm_planes(pa, pb, ta, tb, scratch, bias, epi, beta, ksplit=s, variant=v):
                    t = _bench(lambda: gemm_planes(pa, pb, ta, tb, scratch, bias, epi, beta, ksplit=s, variant=v))
                    best = (t, v, s) if best is None or t < best[0] else best
        if best is None:
            return None
        c = ("hip", round(best[0], 4), None, best[2], best[1])
        GEMM_CHOICES[key] = c
    if c is None:
        return out if gemm_planes(pa, pb, ta, tb, out, bias, epi, beta, ksplit=ks) else None
    return out if gemm_planes(pa, pb, ta, tb, out, bias, epi, beta, ksplit=c[3], variant=c[4]) else None


def _dims(a, b, ta, tb):
    M = a.shape[1] if ta else a.shape[0]
    K = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    return M, N, K


def _hip_ok(a, b, out, *extra):
    ts = (a, b, out) + tuple(t for t in extra if t is not None)
    return all(t.is_cuda and t.dtype == torch.float32 for t in ts) and a.stride(1) == 1 and b.stride(1) == 1 \
        and out.stride(1) == 1


def _hip_gemm(a, b, ta, tb, out, bias=None, epi=EPI_NONE, beta=0.0, aux=None, part=None, colsum=None,
              colsum_acc=False, tile=-1, fp32=None, ksplit=0, dims=None, valid=None, amax=None, amax_out=None):
    """Launch the HIP kernel; returns False (nothing launched) if the shape is not served.

    ``fp32`` picks the product engine (default: the HETSEQ_FP32_GEMM policy); ``ksplit``
    0 = automatic split-K for the split engines, 1 = none, >1 forced.  ``dims`` /
    ``valid``: (M, N, K) of a padded problem and its valid extents (split engines only):
    operand rows past the valid extents read as zero, C rows past valid M are not written.
    ``amax`` = (a's, b's) |max| partials (1-D fp32 device tensors of 1..8 values, or None: computed
    here) for the h3 engine; ``amax_out``: a zeroed 1-element tensor the GELU / dGELU epilogues
    max |C| into.
    """
    M, N, K = dims if dims is not None else _dims(a, b, ta, tb)
    mv, nv, kv = valid if valid is not None else (0, 0, 0)
    assert dims is not None or out.shape == (M, N)
    dt = _FP32_DT[fp32 or _FP32]
    if dt == 4:
        _h3_census((M, N, K, ta, tb, epi), a, b)
    am, keep = (0, 0, 0, 0), []
    if dt == 4:
        am = _amax_ptr(a, amax[0] if amax is not None else None, keep) + _amax_ptr(
            b, amax[1] if amax is not None else None, keep)
    slab = _slab(M, N, ksplit, a.device) if (dt or ksplit > 1) and epi <= EPI_BIAS and ksplit != 1 else None
    rc = hip().gemm(dt, int(ta), int(tb), M, N, K, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                    out.data_ptr(), out.stride(0), bias.data_ptr() if bias is not None else 0, epi, float(beta),
                    aux.data_ptr() if aux is not None else 0, aux.stride(0) if aux is not None else 0,
                    part.data_ptr() if part is not None else 0, colsum.data_ptr() if colsum is not None else 0,
                    int(colsum_acc), stream_handle(), tile, ksplit,
                    slab.data_ptr() if slab is not None else 0, slab.numel() if slab is not None else 0, mv, nv, kv,
                    am[0], am[1], am[2], am[3], slot_ptr(amax_out))
    return rc == 0


def _blas_gemm(a, b, ta, tb, out, bias=None, epi=EPI_NONE, beta=0.0, out_dtype=None):
    A = a.t() if ta else a
    B = b.t() if tb else b
    if out_dtype is not None and out_dtype != A.dtype:
        # library GEMM with bf16 inputs and an fp32 C/D (beta=1 accumulates in place)
        if beta != 0.0:
            torch.ops.aten.addmm.dtype_out(out, A, B, out_dtype, beta=beta, out=out)
        else:
            torch.ops.aten.mm.dtype_out(A, B, out_dtype, out=out)
        if bias is not None and epi >= 1:
            out.add_(bias)
        return out
    if beta != 0.0:
        out.addmm_(A, B, beta=beta)
        if bias is not None and epi >= 1:
            out.add_(bias)
    elif bias is not None and epi >= 1:
        torch.addmm(bias.to(A.dtype), A, B, out=out)
    else:
        torch.mm(A, B, out=out)
    return out


def _bench(fn, iters=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def _choose(key, run_hip, run_blas):
    """The engine of a call site: the hand-written kernels, or the library ORACLE in 'blas' mode."""
    return "blas" if _MODE == "blas" else "hip"


def gemm(a, b, ta=False, tb=False, out=None, bias=None, epi=EPI_NONE, beta=0.0, out_dtype=None, ksplit=None,
         amax=None):
    """out = beta*out + op(a) @ op(b) (+bias).  ``ksplit`` overrides the measured split-K of the HIP engine.
    ``amax``: (a's, b's) |max| partials for the h3 engine (None entries are computed).

    bf16 operands (:class:`Planes` or bf16 matrices) run on the bf16-plane engine (gemm_planes.hip)
    or the library, per measured call site; fp32 tensors on the in-kernel-split engine (gemm.hip) or
    the library."""
    M, N, K = _dims(a, b, ta, tb)
    pa, pb = _as_planes(a), _as_planes(b)
    if pa is not None and pb is not None and _MODE != "blas":
        odt = out_dtype or torch.bfloat16
        if out is None:
            out = torch.empty((M, N), dtype=odt, device=pa.device)
        ks = ksplit if ksplit is not None else (_planes_ksplit(M, N, K, pa.P) if ta and epi == EPI_NONE
                                                and out.dtype == torch.float32 else 1)
        if _bf16_choice((M, N, K, ta, tb, epi, beta != 0.0, "bf16"), pa, pb, ta, tb, out, bias, epi, beta, ks,
                        out_dtype) is not None:
            return out
        a, b = _unplane(a), _unplane(b)  # a shape the plane engine does not serve, or the library
    odt = out_dtype or a.dtype
    if out is None:
        out = torch.empty((M, N), dtype=odt, device=a.device)
    if a.is_cuda and _MODE != "blas" and _hip_ok(a, b, out, bias):
        key = (M, N, K, ta, tb, epi, beta != 0.0)
        scratch = None
        ks = [0]  # split-K of the HIP engine: 0 = kernel heuristic, else measured (auto mode)

        if _FP32 in ("h3", "h3p") and amax is None:  # one |max| pass per operand, shared by the measuring runs
            amax = (amax_of(a), amax_of(b))

        def run_hip():
            return _hip_gemm(a, b, ta, tb, scratch, bias, epi, beta, ksplit=ks[0], amax=amax)

        def run_blas():
            _blas_gemm(a, b, ta, tb, scratch, bias, epi, beta, out_dtype)

        if (key not in GEMM_CHOICES and _MODE == "hip" and _FP32 != "native" and epi <= EPI_BIAS
                and not torch.cuda.is_current_stream_capturing()):
            # the split engines: measure the kernel's own K split once (wave quantisation vs slab traffic)
            scratch = out.clone() if beta != 0.0 else torch.empty_like(out)
            best = None
            for cand in (0, 1, 2, 4):
                ks[0] = cand
                if run_hip():
                    t = _bench(run_hip)
                    if best is None or t < best[0]:
                        best = (t, cand)
            if best is not None:
                ks[0] = best[1]
                GEMM_CHOICES[key] = ("hip", round(best[0], 4), None, best[1])
        c = GEMM_CHOICES.get(key)
        if c is not None and len(c) > 3:
            ks[0] = c[3]
        if ksplit is not None:
            ks[0] = ksplit
        if _choose(key, run_hip, run_blas) == "hip" and _hip_gemm(a, b, ta, tb, out, bias, epi, beta, ksplit=ks[0],
                                                                  amax=amax):
            return out
    return _blas_gemm(a, b, ta, tb, out, bias, epi, beta, out_dtype)


# ------------------------------------------------------------------ tied MLM decoder (V = 30522)
def _pad_vocab(n):
    # a multiple of 512: 128-wide tiles for the logits / weight-gradient products, and K-splits
    # of up to 16 slices for the data-gradient product (K = vocab, only 30 output tiles)
    return (n + 511) // 512 * 512


def _padded_ok(*ts):
    return (_MODE != "blas" and _FP32 != "native" and all(t.is_cuda and t.dtype == torch.float32 for t in ts)
            and ts[0].shape[0] % 128 == 0)


def decoder_logits(t2, w, bias, amax=None):
    """logits [R, V] = t2 [R, H] @ w[V, H]^T + bias, returned as a view of a [R, pad512(V)]
    buffer whose pad columns are zero -- the split-bf16 engine runs the padded problem with the
    missing weight rows / bias entries read as zero.  Library GEMM when faster or not served."""
    R, H = t2.shape
    V = w.shape[0]
    if not _padded_ok(t2, w, bias):
        return gemm(t2, w, tb=True, bias=bias, epi=EPI_BIAS, out_dtype=torch.float32), None
    Vp = _pad_vocab(V)
    buf = torch.empty((R, Vp), dtype=torch.float32, device=t2.device)
    key = (R, V, H, "decoder_fwd")

    if _FP32 in ("h3", "h3p") and amax is None:
        amax = (amax_of(t2), amax_of(w))

    def run_hip():
        return _hip_gemm(t2, w, False, True, buf, bias, EPI_BIAS, 0.0, dims=(R, Vp, H), valid=(R, V, H), amax=amax)

    def run_blas():
        buf[:, V:].zero_()
        torch.addmm(bias, t2, w.t(), out=buf[:, :V])

    if _choose_padded(key, run_hip, run_blas) == "hip" and run_hip():
        return buf[:, :V], buf
    run_blas()
    return buf[:, :V], buf


def decoder_dgrad(dlogits_buf, w, V, amax=None):
    """dt2 [R, H] = dlogits [R, V] @ w [V, H] from the zero-padded [R, pad512(V)] buffer."""
    R, Vp = dlogits_buf.shape
    H = w.shape[1]
    out = torch.empty((R, H), dtype=torch.float32, device=w.device)
    key = (R, H, V, "decoder_dgrad")
    ks = [0]
    if _FP32 in ("h3", "h3p") and amax is None:
        amax = (amax_of(dlogits_buf), amax_of(w))

    def run_hip():
        return _hip_gemm(dlogits_buf, w, False, False, out, dims=(R, H, Vp), valid=(R, H, V), ksplit=ks[0],
                         amax=amax)

    def run_blas():
        torch.mm(dlogits_buf[:, :V], w, out=out)

    if key not in GEMM_CHOICES and _MODE == "hip" and not torch.cuda.is_current_stream_capturing():
        best = None  # K = vocab over only (R/128) x (H/128) tiles: measure the split
        for cand in (4, 8, 16):
            ks[0] = cand
            if run_hip():
                t = _bench(run_hip)
                best = (t, cand) if best is None or t < best[0] else best
        if best is not None:
            GEMM_CHOICES[key] = ("hip", round(best[0], 4), None, best[1])
    c = GEMM_CHOICES.get(key)
    if c is not None and len(c) > 3:
        ks[0] = c[3]
    if _choose_padded(key, run_hip, run_blas) == "hip" and run_hip():
        return out
    run_blas()
    return out


def decoder_wgrad(dlogits_buf, t2, V, out, accumulate, amax=None):
    """dW [V, H] (+)= dlogits^T @ t2 from the zero-padded buffer (rows past V are not written)."""
    R, Vp = dlogits_buf.shape
    H = t2.shape[1]
    key = (V, H, R, "decoder_wgrad", bool(accumulate))
    beta = 1.0 if accumulate else 0.0
    if _FP32 in ("h3", "h3p") and amax is None:
        amax = (amax_of(dlogits_buf), amax_of(t2))

    def run_hip(dst):
        return _hip_gemm(dlogits_buf, t2, True, False, dst, beta=beta, dims=(Vp, H, R), valid=(V, H, R), amax=amax)

    def run_blas(dst):
        if accumulate:
            dst.addmm_(dlogits_buf[:, :V].t(), t2)
        else:
            torch.mm(dlogits_buf[:, :V].t(), t2, out=dst)

    if _choose_padded(key, None, None) == "hip" and run_hip(out):
        return out
    run_blas(out)
    return out


def decoder_wgrad_bf16(dl_p, t2, V, out, accumulate):
    """bf16 engine: dW [V, H] (+)= dlogits^T @ t2 with dlogits the zero-padded [R, pad512(V)] bf16 copy
    of the loss gradient -- the plane kernels over the padded rows, C rows past V neither read nor
    written (fp32 ``out``).  The library (``torch.mm``) in 'blas' mode or for a shape not served."""
    beta = 1.0 if accumulate else 0.0
    if _MODE != "blas":
        pa, pb = _as_planes(dl_p), _as_planes(t2)
        if pa is not None and pb is not None:
            Vp, H, R = dl_p.shape[1], t2.shape[1], t2.shape[0]
            if gemm_planes(pa, pb, True, False, out, beta=beta, ksplit=_planes_ksplit(Vp, H, R, 1), mv=V):
                return out
    prod = torch.mm(dl_p[:, :V].t(), t2).float()
    return out.add_(prod) if accumulate else out.copy_(prod)


def _choose_padded(key, run_hip, run_blas):
    """Engine of the padded decoder products: the hand-written kernels (the library in 'blas' mode)."""
    return _choose(key, run_hip, run_blas)


def linear_fwd(x, w, bias=None, out=None, ksplit=None, amax=None):
    """x[T,K] @ w[N,K]^T (+bias)."""
    return gemm(x, w, ta=False, tb=True, out=out, bias=bias, epi=EPI_BIAS if bias is not None else EPI_NONE,
                ksplit=ksplit, amax=amax)


def linear_fwd_partials(x, w, ksplit=None, amax=None):
    """x[T,K] @ w[N,K]^T for a consumer that sums split-K partials itself (the LN forward after the
    FFN-out product): ``(partials [ks, T, N], ks)`` with the split-bf16 engine's K slices left in the
    stream's slab -- no reduce pass, the LN reads the slices in the reduce kernel's order, so the
    result is bitwise the same -- or ``(out, 1)`` from any other path (first, measuring call;
    library choice; plane operands).  The view aliases the slab: consume it before the next GEMM
    on this stream."""
    M, K = x.shape
    N = w.shape[0]
    if (_MODE != "blas" and _FP32 != "native" and x.is_cuda and isinstance(x, torch.Tensor)
            and isinstance(w, torch.Tensor) and _hip_ok(x, w, x)):
        c = GEMM_CHOICES.get((M, N, K, False, True, EPI_NONE, False))
        if c is not None and c[0] == "hip":
            ks = ksplit if ksplit is not None else (c[3] if len(c) > 3 else 0)
            slab = _slab(M, N, ks, x.device)
            if slab is not None:
                am, keep = (0, 0, 0, 0), []
                _h3_census((M, N, K, 0, 1, 0), x, w)
                if _FP32 in ("h3", "h3p"):
                    am = _amax_ptr(x, amax[0] if amax is not None else None, keep) + _amax_ptr(
                        w, amax[1] if amax is not None else None, keep)
                rc = hip().gemm(_FP32_DT[_FP32], 0, 1, M, N, K, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0),
                                0, N, 0, EPI_NONE, 0.0, 0, 0, 0, 0, 0, stream_handle(), -1, ks, slab.data_ptr(),
                                slab.numel(), 0, 0, 0, am[0], am[1], am[2], am[3], 0)
                if rc == 0:
                    n = hip().gemm_last_ksplit()
                    return slab[:n * M * N].view(n, M, N), n
    return linear_fwd(x, w, amax=amax), 1


def linear_dgrad(dy, w, out=None, accumulate=False, ksplit=None, amax=None):
    """dy[T,N] @ w[N,K]; accumulate=True adds into ``out``."""
    return gemm(dy, w, ta=False, tb=False, out=out, beta=1.0 if accumulate else 0.0, ksplit=ksplit, amax=amax)


def linear_wgrad(dy, x, out=None, accumulate=False, ksplit=None, amax=None):
    """dy[T,N]^T @ x[T,K] -> [N,K] in fp32; accumulate=True adds into ``out`` (flat grad view)."""
    return gemm(dy, x, ta=True, tb=False, out=out, out_dtype=torch.float32, beta=1.0 if accumulate else 0.0,
                ksplit=ksplit, amax=amax)


def linear_wgrad_colsum(dy, x, out, colsum_out, ksplit=None, accumulate=True, amax=None):
    """``out (+)= dy^T @ x`` and ``colsum_out (+)= dy.sum(0)`` (a Linear's weight and bias gradients) in
    one split-bf16 launch: the weight-gradient blocks of the first column tile sum dy's columns from
    the registers they stage (gemm.hip, ``wcol``), and one small pass adds the K slices' partials
    into ``colsum_out``.  Returns False when not served (library choice, first measuring call, other
    layouts): the caller then runs :func:`linear_wgrad` and a column sum."""
    T, M = dy.shape
    N = x.shape[1]
    if not (_MODE != "blas" and _FP32 in SPLIT_ENGINES and isinstance(dy, torch.Tensor) and isinstance(x, torch.Tensor)
            and dy.is_cuda and dy.dtype == torch.float32 and x.dtype == torch.float32 and out.is_contiguous()
            and colsum_out.is_contiguous() and colsum_out.numel() == M and _hip_ok(dy, x, out)):
        return False
    # the same engine decision as linear_wgrad's (so a run takes the fused path from its first step
    # on, whatever the choice table held: the bias gradient's summation order never switches)
    key = (M, N, T, True, False, EPI_NONE, True)
    ks = ksplit if ksplit is not None else 0
    if key not in GEMM_CHOICES:
        if torch.cuda.is_current_stream_capturing():
            return False
        gemm(dy, x, ta=True, tb=False, out=torch.empty_like(out), beta=1.0, out_dtype=torch.float32,
             ksplit=ksplit, amax=amax)  # first call: measures the kernel's K split (into scratch)
    c = GEMM_CHOICES.get(key)
    if c is None or c[0] != "hip":
        return False
    if ksplit is None and len(c) > 3:
        ks = c[3]
    part = torch.empty((max(ks, 1) if ks > 0 else 8, M), dtype=torch.float32, device=dy.device)
    return _hip_gemm(dy, x, True, False, out, beta=1.0 if accumulate else 0.0, part=part, colsum=colsum_out,
                     colsum_acc=accumulate, ksplit=ks, amax=amax)


def linear_gelu_fwd(x, w, b, out=None, amax=None, amax_out=None):
    """FFN-in forward: pre = x @ w^T (un-biased, kept for the backward), y = gelu(pre + b).

    Returns (y, pre).  One fused HIP GEMM (epilogue writes both) or library GEMM + bias_gelu kernel.
    ``out`` = (y, pre) buffers to write (fp32 operands; row slices of whole-batch tensors).
    ``amax``: (x's, w's) |max| partials (h3 engine); ``amax_out``: a zeroed 1-element tensor that
    receives |max| of y (the FFN-out product's operand scale) -- filled on every path.
    """
    from hetseq_amd.ops import bert_ops

    T, N = x.shape[0], w.shape[0]
    px, pw = _as_planes(x), _as_planes(w)
    if px is not None and pw is not None and _MODE != "blas":  # bf16 operands
        if out is not None and all(t.dtype == torch.bfloat16 for t in out):
            y, pre = out  # (row slices of whole-batch tensors: the half-batch forward chains)
        else:
            pre = torch.empty((T, N), dtype=torch.bfloat16, device=px.device)
            y = torch.empty_like(pre)
        if gemm_planes(px, pw, False, True, y, b, EPI_GELU, 0.0, aux=pre):
            return y, pre
        x, w = _unplane(x), _unplane(w)
    if out is not None:
        y, pre = out
    else:
        pre = torch.empty((T, N), dtype=x.dtype, device=x.device)
        y = torch.empty_like(pre)
    if x.is_cuda and _MODE != "blas" and _hip_ok(x, w, y, b, pre):
        key = (T, N, x.shape[1], "gelu_fwd")
        if _FP32 in ("h3", "h3p") and amax is None:
            amax = (amax_of(x), amax_of(w))

        def run_hip(amo=None):
            return _hip_gemm(x, w, False, True, y, b, EPI_GELU, 0.0, aux=pre, amax=amax, amax_out=amo)

        def run_blas():
            torch.mm(x, w.t(), out=pre)
            bert_ops.bias_gelu_fwd(pre, b, out=y)

        if _choose(key, run_hip, run_blas) == "hip" and run_hip(amax_out):
            return y, pre
    torch.mm(x, w.t(), out=pre)
    bert_ops.bias_gelu_fwd(pre, b, out=y)
    if amax_out is not None:
        amax_into(y, amax_out)
    return y, pre


def linear_dgrad_dgelu(dy, w, pre, b, db_acc=None, amax=None, amax_out=None, colsum=True):
    """FFN backward through the GELU: dpre = (dy @ w) * gelu'(pre + b), db = colsum(dpre).

    ``db`` is accumulated into ``db_acc`` (flat-store view) when given.  Returns (dpre, db);
    ``colsum=False`` (HIP engine only; else ignored): no db -- returns (dpre, None), the caller sums
    the bias gradient elsewhere (bert_ops: inside the FFN-in weight-gradient launch).
    ``amax`` / ``amax_out``: as in :func:`linear_gelu_fwd` (|max| of dpre into ``amax_out``).
    """
    from hetseq_amd.ops import bert_ops

    T, N = dy.shape[0], w.shape[1]
    db = db_acc if db_acc is not None else torch.empty(N, dtype=torch.float32, device=dy.device)
    pd, pw = _as_planes(dy), _as_planes(w)
    if pd is not None and pw is not None and _MODE != "blas":  # bf16 operands
        part = torch.empty(((T + 127) // 128, N), dtype=torch.float32, device=pre.device)
        dpre = torch.empty((T, N), dtype=pre.dtype, device=pre.device)
        if gemm_planes(pd, pw, False, False, dpre, b, EPI_DGELU, 0.0, aux=pre, part=part, colsum=db,
                       colsum_acc=db_acc is not None):
            return dpre, db
        dy, w = _unplane(dy), _unplane(w)
    dpre = torch.empty((T, N), dtype=dy.dtype, device=dy.device)
    if dy.is_cuda and _MODE != "blas" and _hip_ok(dy, w, dpre, pre, b):
        key = (T, N, dy.shape[1], "dgelu")
        part = torch.empty(((T + 63) // 64, N), dtype=torch.float32, device=dy.device)
        if _FP32 in ("h3", "h3p") and amax is None:
            amax = (amax_of(dy), amax_of(w))

        def run_hip(out_db, acc, amo=None):
            return _hip_gemm(dy, w, False, False, dpre, b, EPI_DGELU, 0.0, aux=pre,
                             part=part if out_db is not None else None, colsum=out_db, colsum_acc=acc, amax=amax,
                             amax_out=amo)

        if _choose(key, None, None) == "hip" and run_hip(db if colsum else None, db_acc is not None, amax_out):
            return dpre, (db if colsum else None)
    df = torch.mm(dy, w)
    dpre, db = bert_ops.gelu_bwd_colsum(df, pre, b, db_acc=db_acc)
    if amax_out is not None:
        amax_into(dpre, amax_out)
    return dpre, db


# ------------------------------------------------------------------ h3 operand scales per forward
_SEG_TABLES: dict = {}  # (device, ((ptr, numel), ...)) -> (base ptr, int64 [nblk, 3] table, nblk)
_SEG_CHUNK4 = 2048  # float4s per amax_seg block (8 Ki floats; tools/bench_amax.py: 71 vs 77 us at 16384)


def _seg_table(ts):
    """Block table of ``amax_seg`` over the fp32 tensors ``ts`` (each contiguous, 16-B aligned,
    numel % 4 == 0): offsets are float4 indices from the lowest address, so separate allocations
    (no flat store) work as well as views into one flat buffer."""
    dev = ts[0].device
    key = (dev, tuple((t.data_ptr(), t.numel()) for t in ts))
    hit = _SEG_TABLES.get(key)
    if hit is not None:
        return hit
    base = min(t.data_ptr() for t in ts)
    rows = []
    for i, t in enumerate(ts):
        assert t.dtype == torch.float32 and t.is_contiguous() and t.numel() % 4 == 0 and t.data_ptr() % 16 == 0
        lo = (t.data_ptr() - base) // 16
        hi = lo + t.numel() // 4
        for c in range(lo, hi, _SEG_CHUNK4):
            rows.append((i, c, min(hi, c + _SEG_CHUNK4)))
    tab = torch.tensor(rows, dtype=torch.int64, device=dev)
    hit = (base, tab, len(rows))
    if len(_SEG_TABLES) > 64:
        _SEG_TABLES.clear()
    _SEG_TABLES[key] = hit
    return hit


# weight |max| of all but the first layer measured on the weight-gradient stream (idle at the start
# of the forward) beside the first layer's work
_SPLIT_WEIGHT_AMAX = True
_REST_EVENTS: dict = {}


def _rest_event(device):
    ev = _REST_EVENTS.get(device)
    if ev is None:
        ev = _REST_EVENTS[device] = torch.cuda.Event()
    return ev


class AmaxPool(object):
    """|max| slots of one forward + backward on the h3 engine (zeroed once, 1 launch):

    * ``w(i)``: weight ``i`` of the list given at construction -- filled right away by ONE
      ``amax_seg`` launch over all of them (weights change in place every update, so every forward
      measures them again; ~50 us for BERT-base's 86 M GEMM weights); a None entry reserves its
      slot unmeasured;
    * ``act(i, n)``: activation / gradient slots, atomically maxed by the kernels that produce
      those tensors (LN forward / backward, GELU / dGELU epilogues, embedding) or by ``amax_of``.
    Each slot has exactly one producer stream, and its consumers are ordered after that producer,
    so the scales -- and the results -- are deterministic."""

    def __init__(self, weights, n_act, device, split=0):
        self.nw = len(weights)
        self.buf = torch.zeros((self.nw + n_act) * SLOT_FLOATS, dtype=torch.float32, device=device)
        self.ptr = self.buf.data_ptr()
        self.rest = None
        from hetseq_amd.runtime import streams

        self._deferred = None
        first = next((i for i, w in enumerate(weights) if w is not None), len(weights))
        if first > 0:  # leading reserved slots (h3p engine layers): the rest is measured by
            rest = [w for w in weights[first:]]  # measure_deferred(), just before its consumer
            if rest and all(w is not None for w in rest):
                self._deferred = (_seg_table(rest), first)
            return
        if 0 < split < len(weights) and _SPLIT_WEIGHT_AMAX and streams.enabled() and self.buf.is_cuda:
            # weights [0, split) now; the rest on the side stream, beside the first layer's work
            # (consumers on the current stream call wait_rest() first; the side stream's own later
            # work is ordered after it)
            base, tab, nblk = _seg_table(weights[:split])
            hip().amax_seg(base, tab.data_ptr(), nblk, self.ptr, stream_handle())
            base, tab, nblk = _seg_table(weights[split:])
            st = streams.side(self.buf.device)
            hip().stream_wait(st.cuda_stream, stream_handle())
            hip().amax_seg(base, tab.data_ptr(), nblk, self.ptr + 4 * SLOT_FLOATS * split, st.cuda_stream)
            self.rest = _rest_event(self.buf.device)
            self.rest.record(st)
        elif weights:
            base, tab, nblk = _seg_table(weights)
            hip().amax_seg(base, tab.data_ptr(), nblk, self.ptr, stream_handle())

    def measure_deferred(self):
        """Measure the weights after the leading reserved slots (the pre-training head's), on the
        current stream -- called by their consumer once they are current (a staged update)."""
        if self._deferred is not None:
            (base, tab, nblk), first = self._deferred
            self._deferred = None
            hip().amax_seg(base, tab.data_ptr(), nblk, self.ptr + 4 * SLOT_FLOATS * first, stream_handle())

    def wait_rest(self):
        """The current stream waits for the side-stream part of the weight |max| (no-op without one)."""
        if self.rest is not None:
            torch.cuda.current_stream(self.buf.device).wait_event(self.rest)
            self.rest = None

    # slots are (pointer, count) tuples: plain ints, so the ~150 uses per step cost no tensor views
    def w(self, i):
        return (self.ptr + 4 * SLOT_FLOATS * i, 1)

    def act(self, i, n=1):
        return (self.ptr + 4 * SLOT_FLOATS * (self.nw + i), n)

    def value(self, slot):
        """|max| held by a slot (diagnostics; host sync)."""
        i = (slot[0] - self.ptr) // (4 * SLOT_FLOATS)
        return amax_value(self.buf[i * SLOT_FLOATS:(i + slot[1]) * SLOT_FLOATS]).max().item()


def h3_active(dtype=torch.float32):
    """True when fp32 GEMMs run on the h3 engine (operand |max| slots are worth tracking)."""
    return _FP32 in ("h3", "h3p") and _MODE != "blas" and dtype == torch.float32


def h3p_active(dtype=torch.float32):
    """True when the encoder layers' fp32 products run on the h3p plane engine (ops/h3p.py)."""
    return _FP32 == "h3p" and _MODE != "blas" and dtype == torch.float32
