"""GEMM dispatch for the BERT hot path.

``linear_fwd`` / ``linear_dgrad`` / ``linear_wgrad`` are the three products
of a Linear layer.  Two engines:

* ``hip``  -- the hand-written gfx950 MFMA kernel (csrc/kernels/gemm.hip) with
             fused epilogues (bias, bias+GELU, beta-accumulate); fp32 today.
* ``blas`` -- hipBLASLt through ``torch.addmm`` (plain library GEMM).

``HETSEQ_GEMM=hip|blas|auto`` selects; ``auto`` (default) times both engines
once per (shape, transpose, dtype) on the GPU and keeps the faster one --
the choice is recorded in ``GEMM_CHOICES`` and logged by the benchmark.
In bf16 mode the weight-gradient GEMM writes fp32 directly (``out_dtype``),
so master gradients never round through bf16.
"""
from __future__ import annotations

import os

import torch

from hetseq_amd.ops._C import hip, stream_handle

GEMM_CHOICES: dict = {}
_MODE = os.environ.get("HETSEQ_GEMM", "auto")


def set_mode(mode):
    global _MODE
    assert mode in ("hip", "blas", "auto")
    _MODE = mode
    GEMM_CHOICES.clear()


def _hip_gemm(a, b, ta, tb, out, bias=None, epi=0, beta=0.0):
    M = a.shape[1] if ta else a.shape[0]
    K = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    assert out.shape == (M, N) and out.is_contiguous() and a.stride(1) == 1 and b.stride(1) == 1
    hip().gemm(0, int(ta), int(tb), M, N, K, a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), out.data_ptr(),
               out.stride(0), bias.data_ptr() if bias is not None else 0, epi, float(beta), stream_handle())
    return out


def _blas_gemm(a, b, ta, tb, out, bias=None, epi=0, beta=0.0, out_dtype=None):
    A = a.t() if ta else a
    B = b.t() if tb else b
    if out_dtype is not None and out_dtype != A.dtype:
        if beta != 0.0:
            out.add_(torch.mm(A, B, out_dtype=out_dtype))
        else:
            res = torch.mm(A, B, out_dtype=out_dtype)
            out.copy_(res)
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


def _choose(key, a, b, ta, tb, out, bias, epi, beta):
    if _MODE != "auto":
        return _MODE
    c = GEMM_CHOICES.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return "blas"
        scratch = torch.empty_like(out)
        if beta != 0.0:
            scratch.copy_(out)
        t_hip = _bench(lambda: _hip_gemm(a, b, ta, tb, scratch, bias, epi, beta))
        t_blas = _bench(lambda: _blas_gemm(a, b, ta, tb, scratch, bias, epi, beta))
        c = "hip" if t_hip < t_blas else "blas"
        GEMM_CHOICES[key] = (c, round(t_hip, 4), round(t_blas, 4))
        return c
    return c[0]


def gemm(a, b, ta=False, tb=False, out=None, bias=None, epi=0, beta=0.0, out_dtype=None):
    """out = beta*out + op(a) @ op(b) (+bias) (gelu if epi == 2, hip engine only)."""
    M = a.shape[1] if ta else a.shape[0]
    N = b.shape[0] if tb else b.shape[1]
    odt = out_dtype or a.dtype
    if out is None:
        out = torch.empty((M, N), dtype=odt, device=a.device)
    hip_ok = (a.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32 and out.dtype == torch.float32
              and a.stride(1) == 1 and b.stride(1) == 1 and out.is_contiguous())
    if epi == 2 and not hip_ok:
        raise RuntimeError("fused GELU epilogue needs the fp32 HIP GEMM")
    if a.is_cuda and hip_ok:
        key = (M, N, a.shape[0] if ta else a.shape[1], ta, tb, epi, beta != 0.0)
        if epi == 2 or _choose(key, a, b, ta, tb, out, bias, epi, beta) == "hip":
            return _hip_gemm(a, b, ta, tb, out, bias, epi, beta)
    return _blas_gemm(a, b, ta, tb, out, bias, epi, beta, out_dtype)


def linear_fwd(x, w, bias=None, out=None):
    """x[T,K] @ w[N,K]^T (+bias)."""
    return gemm(x, w, ta=False, tb=True, out=out, bias=bias, epi=1 if bias is not None else 0)


def linear_dgrad(dy, w, out=None, accumulate=False):
    """dy[T,N] @ w[N,K]; accumulate=True adds into ``out``."""
    return gemm(dy, w, ta=False, tb=False, out=out, beta=1.0 if accumulate else 0.0)


def linear_wgrad(dy, x, out=None, accumulate=False):
    """dy[T,N]^T @ x[T,K] -> [N,K] in fp32; accumulate=True adds into ``out`` (flat grad view)."""
    return gemm(dy, x, ta=True, tb=False, out=out, out_dtype=torch.float32, beta=1.0 if accumulate else 0.0)
