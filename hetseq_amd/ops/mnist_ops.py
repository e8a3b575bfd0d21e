"""MNISTNet forward / backward on the gfx950 kernels (K15; csrc/kernels/mnist.hip).

Reference: tasks.py:337-362 (the PyTorch MNIST example network) and eval_mnist.py:9-37.  One
autograd Function runs the whole network: conv1 (direct kernel), conv2 as an implicit GEMM over an
im2col matrix on the exact-fp32 MFMA engine (``ops.gemm`` native), the fused
ReLU / 2x2-max / Dropout2d pooling stage, fc1 on the same GEMM engine, and one fused
ReLU + dropout + fc2 + log_softmax + NLL kernel; the backward mirrors it (the im2col transpose is
a fixed-order gather: no atomics, bitwise reproducible).  fp32 throughout, as the reference.

The fc activations are padded to a multiple of 64 rows (zero rows) and the conv2 GEMM rows (B x 576
pixels) to a multiple of 2048 so every GEMM tiles exactly and the deep-K weight-gradient products
split K (``_ks``; the split-K partials are summed in a fixed order, so the result is deterministic).
Activations are channel-last and fc1's weight columns are permuted to the pooled (y, x, c) order,
so every gather and scatter around the GEMMs is a contiguous run.
"""
from __future__ import annotations

import torch

from hetseq_amd.ops import gemm as G
from hetseq_amd.ops._C import hip, stream_handle
from hetseq_amd.runtime import rng

KP = 320  # conv2 reduction length (9 x 32 = 288) padded to a multiple of 64
ROWS = 2048  # conv2 GEMM rows (B*576 pixels) are padded to a multiple of 64 K-slices x 32
WG_PART = 1024 * 320  # weight-gradient scratch: conv1 (mnist.hip kWgChunks x 320) >= fc2 (64 x 1290)


def _ks(M, N, K):
    """Split-K for a small output with a deep K: slices until the 64x64 tiles fill ~512 blocks."""
    tiles, ks = max(1, (M // 64) * (N // 64)), 1
    while tiles * ks * 2 <= 512 and K % (ks * 2 * 32) == 0 and K // (ks * 2) >= 256:
        ks *= 2
    return ks


def _mm(a, b, ta, tb, out, bias=None):
    """Exact-fp32 MFMA GEMM (gemm.hip); the padded shapes here are always served."""
    M, N = out.shape
    K = a.shape[0] if ta else a.shape[1]
    ok = G._hip_gemm(a, b, ta, tb, out, bias, G.EPI_BIAS if bias is not None else G.EPI_NONE, 0.0, fp32="native",
                     ksplit=_ks(M, N, K))
    if not ok:
        raise RuntimeError("MNIST GEMM shape not served by the HIP engine: %s x %s" % (tuple(a.shape), tuple(b.shape)))
    return out


def _perm(src, rows, cols, mode):
    """Column permutations of the weights (mnist.hip perm_cols_kernel): 0 conv2 filter -> padded
    (ky, kx, ci) columns, 1 its inverse, 2 fc1 columns (c, y, x) -> (y, x, c), 3 its inverse."""
    dst = torch.empty((rows, cols), dtype=torch.float32, device=src.device)
    hip().mnist_perm(src.data_ptr(), dst.data_ptr(), rows, mode, stream_handle())
    return dst


class FusedMNIST(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target, wc1, bc1, wc2, bc2, w1, b1, w2, b2, p1, p2, mean):
        B = x.shape[0]
        Bp = (B + 63) // 64 * 64
        R = (B * 576 + ROWS - 1) // ROWS * ROWS
        dev = x.device
        x = x.contiguous().float()
        target = target.contiguous()
        st = stream_handle()
        h1 = torch.empty((B, 26, 26, 32), dtype=torch.float32, device=dev)  # NHWC
        hip().mnist_conv1_fwd(x.data_ptr(), wc1.data_ptr(), bc1.data_ptr(), h1.data_ptr(), B, st)
        col = torch.empty((R, KP), dtype=torch.float32, device=dev)
        hip().mnist_im2col(h1.data_ptr(), col.data_ptr(), B, R, st)
        wp = _perm(wc2.contiguous(), 64, KP, 0)
        c2 = _mm(col, wp, False, True, torch.empty((R, 64), dtype=torch.float32, device=dev), bc2)
        pooled = torch.empty((Bp, 9216), dtype=torch.float32, device=dev)  # (y, x, c) columns
        arg = torch.empty((B, 9216), dtype=torch.uint8, device=dev)
        s1, o1 = rng.fork() if p1 > 0 else (0, 0)
        hip().mnist_pool_fwd(c2.data_ptr(), pooled.data_ptr(), arg.data_ptr(), B, Bp, float(p1), s1, o1, st)
        w1p = _perm(w1.contiguous(), 128, 9216, 2)
        pre = _mm(pooled, w1p, False, True, torch.empty((Bp, 128), dtype=torch.float32, device=dev), b1)
        h = torch.empty((Bp, 128), dtype=torch.float32, device=dev)
        logp = torch.empty((B, 10), dtype=torch.float32, device=dev)
        nll = torch.empty(B, dtype=torch.float32, device=dev)
        s2, o2 = rng.fork() if p2 > 0 else (0, 0)
        hip().mnist_head_fwd(pre.data_ptr(), w2.data_ptr(), b2.data_ptr(), target.data_ptr(), h.data_ptr(),
                             logp.data_ptr(), nll.data_ptr(), B, float(p2), s2, o2, st)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        aux = torch.empty(2, dtype=torch.float32, device=dev)  # correct, count of valid targets
        hip().mnist_loss(nll.data_ptr(), logp.data_ptr(), target.data_ptr(), B, int(mean), loss.data_ptr(),
                         aux[0:1].data_ptr(), aux[1:2].data_ptr(), st)
        ctx.save_for_backward(x, target, h1, col, wp, arg, pooled, pre, h, logp, aux, w1p, w2)
        ctx.cfg = (B, Bp, R, float(p1), float(p2), int(mean))
        ctx.mark_non_differentiable(aux)
        return loss, aux

    @staticmethod
    def backward(ctx, dloss, _daux):
        x, target, h1, col, wp, arg, pooled, pre, h, logp, aux, w1p, w2 = ctx.saved_tensors
        B, Bp, R, p1, p2, mean = ctx.cfg
        dev = x.device
        st = stream_handle()
        dloss = dloss.contiguous().float().reshape(1)
        dlogits = torch.empty((Bp, 10), dtype=torch.float32, device=dev)
        dpre = torch.empty((Bp, 128), dtype=torch.float32, device=dev)
        hip().mnist_head_bwd(dloss.data_ptr(), aux[1:2].data_ptr(), logp.data_ptr(), target.data_ptr(),
                             pre.data_ptr(), h.data_ptr(), w2.data_ptr(), dlogits.data_ptr(), dpre.data_ptr(), B, Bp,
                             mean, p2, st)
        dw2 = torch.empty((10, 128), dtype=torch.float32, device=dev)
        db2 = torch.empty(10, dtype=torch.float32, device=dev)
        part = torch.empty(WG_PART, dtype=torch.float32, device=dev)
        hip().mnist_fc2_wgrad(dlogits.data_ptr(), h.data_ptr(), part.data_ptr(), dw2.data_ptr(), db2.data_ptr(), B,
                              st)
        from hetseq_amd.ops.bert_ops import colsum

        dw1p = _mm(dpre, pooled, True, False, torch.empty((128, 9216), dtype=torch.float32, device=dev))
        dw1 = _perm(dw1p, 128, 9216, 3)
        db1 = colsum(dpre)
        dpooled = _mm(dpre, w1p, False, False, torch.empty((Bp, 9216), dtype=torch.float32, device=dev))
        dc2 = torch.empty((R, 64), dtype=torch.float32, device=dev)
        hip().mnist_pool_bwd(dpooled.data_ptr(), arg.data_ptr(), dc2.data_ptr(), B, R, p1, st)
        dwp = _mm(dc2, col, True, False, torch.empty((64, KP), dtype=torch.float32, device=dev))
        dwc2 = _perm(dwp, 64, 288, 1).view(64, 32, 3, 3)
        dbc2 = colsum(dc2)
        dcol = _mm(dc2, wp, False, False, torch.empty((R, KP), dtype=torch.float32, device=dev))
        dh1 = torch.empty_like(h1)
        hip().mnist_col2im(dcol.data_ptr(), h1.data_ptr(), dh1.data_ptr(), B, st)
        dwc1 = torch.empty((32, 1, 3, 3), dtype=torch.float32, device=dev)
        dbc1 = torch.empty(32, dtype=torch.float32, device=dev)
        hip().mnist_conv1_wgrad(dh1.data_ptr(), x.data_ptr(), part.data_ptr(), dwc1.data_ptr(), dbc1.data_ptr(), B, st)
        return None, None, dwc1, dbc1, dwc2, dbc2, dw1, db1, dw2, db2, None, None, None


def mnist_loss(model, x, target, eval=False):
    """(loss, correct) of MNISTNet on the HIP kernels: mean NLL for training, (sum, #correct) for eval."""
    p1 = model.dropout1.p if model.training else 0.0
    p2 = model.dropout2.p if model.training else 0.0
    loss, aux = FusedMNIST.apply(x, target, model.conv1.weight, model.conv1.bias, model.conv2.weight,
                                 model.conv2.bias, model.fc1.weight, model.fc1.bias, model.fc2.weight,
                                 model.fc2.bias, p1, p2, not eval)
    return loss, aux[0]
