"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 oracle."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref_ln(x, g, b, eps=1e-12):
    u = x.mean(-1, keepdim=True)
    s = (x - u).pow(2).mean(-1, keepdim=True)
    return g * (x - u) / torch.sqrt(s + eps) + b


def _close(a, b, rtol=1e-4, atol=1e-5, msg=""):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, "%s max err %.3e > %.3e" % (msg, err, tol)


@pytest.mark.parametrize("H", [256, 768, 1024])
def test_layernorm_fwd_bwd(cuda, H):
    from hetseq_amd.ops.bert_ops import layer_norm

    torch.manual_seed(0)
    x = torch.randn(300, H, device=cuda, requires_grad=True)
    g = torch.randn(H, device=cuda, requires_grad=True)
    b = torch.randn(H, device=cuda, requires_grad=True)
    y = layer_norm(x, g, b)
    x2, g2, b2 = (t.detach().clone().requires_grad_() for t in (x, g, b))
    y2 = _ref_ln(x2, g2, b2)
    _close(y, y2, msg="ln fwd")
    dy = torch.randn_like(y)
    y.backward(dy)
    y2.backward(dy)
    _close(x.grad, x2.grad, 1e-4, 1e-4, "ln dx")
    _close(g.grad, g2.grad, 1e-4, 1e-3, "ln dgamma")
    _close(b.grad, b2.grad, 1e-4, 1e-3, "ln dbeta")


@pytest.mark.parametrize("T,F_", [(1024, 3072), (2048, 768)])
def test_ffn_out_partials_into_ln_bitwise(cuda, T, F_):
    """FFN-out (K 3072) and attention-output (K 768, the half-batch forward's shape) products with
    their split-K partials summed by the LN forward (no reduce pass) give bitwise the LN of the
    reduced product: same slice order, same bias / dropout / residual."""
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(3)
    H = 768
    x = torch.randn(T, F_, device=cuda)
    w = torch.randn(H, F_, device=cuda) * 0.02
    b = torch.randn(H, device=cuda) * 0.1
    r = torch.randn(T, H, device=cuda)
    g = torch.rand(H, device=cuda) + 0.5
    be = torch.randn(H, device=cuda) * 0.1
    G.linear_fwd(x, w)  # first call measures the engine and K split
    parts, n = G.linear_fwd_partials(x, w)
    if G.GEMM_CHOICES[(T, H, F_, False, True, 0, False)][0] == "hip":
        assert parts.dim() == 3 and parts.shape[1:] == (T, H) and n == parts.shape[0]
    y1, z1, m1, r1 = bert_ops.ln_fwd(parts, g, be, bias=b, resid=r, p=0.1, mode=1, seed=5, off=9)
    y2, z2, m2, r2 = bert_ops.ln_fwd(G.linear_fwd(x, w), g, be, bias=b, resid=r, p=0.1, mode=1, seed=5, off=9)
    assert torch.equal(y1, y2) and torch.equal(z1, z2) and torch.equal(m1, m2) and torch.equal(r1, r2)
    ref = x.double() @ w.double().t()
    _close(parts.sum(0) if parts.dim() == 3 else parts, ref, 1e-5, 1e-5, "partials sum")


@pytest.mark.parametrize("tile", [-1, 512])  # transposed-read A layout (default) / register transpose
@pytest.mark.parametrize("ks", [2, 4])
@pytest.mark.parametrize("acc", [True, False])  # accumulate / store (first backward after zero_grad)
def test_wgrad_colsum_fused(cuda, tile, ks, acc):
    """QKV-shaped weight gradient with the bias gradient summed by the same launch (the first column
    tile's blocks add up the dy columns they stage): dW (+)= dy^T x and db (+)= sum_rows(dy),
    against fp64."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(6)
    T, M, N = 4096, 2304, 768
    dy, x = torch.randn(T, M, device=cuda), torch.randn(T, N, device=cuda)
    w0, c0 = torch.randn(M, N, device=cuda), torch.randn(M, device=cuda)
    w, c = w0.clone(), c0.clone()
    part = torch.empty((ks, M), dtype=torch.float32, device=cuda)
    assert G._hip_gemm(dy, x, True, False, w, beta=1.0 if acc else 0.0, part=part, colsum=c, colsum_acc=acc,
                       fp32="x6", ksplit=ks, tile=tile)
    if not acc:
        w0.zero_()
        c0.zero_()
    d, xd = dy.double(), x.double()
    scale = w0.double().abs() + d.abs().t() @ xd.abs()
    assert float(((w.double() - (w0.double() + d.t() @ xd)).abs() / scale).max()) < 1e-6
    cscale = c0.double().abs() + d.abs().sum(0)
    assert float(((c.double() - (c0.double() + d.sum(0))).abs() / cscale).max()) < 1e-6


def test_ln_bwd_chunked_partials_bitwise(cuda):
    """The LN backward's 3 KB-LDS column partials sum the four waves in the same pairwise order as
    the [waves][H] LDS image: dgamma / dbeta / dbias and dz / da are bitwise equal."""
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops._C import hip

    torch.manual_seed(4)
    rows, H = 4096, 768
    dy, z = torch.randn(rows, H, device=cuda), torch.randn(rows, H, device=cuda)
    mean, rstd = torch.randn(rows, device=cuda), torch.rand(rows, device=cuda) + 0.5
    g = torch.randn(H, device=cuda)
    outs = []
    try:
        for chunked in (1, 0):
            hip().set_ln_bwd_lds(chunked)
            outs.append(bert_ops.ln_bwd(dy, z, mean, rstd, g, 0.1, 1, 1, 2, True, True))
    finally:
        hip().set_ln_bwd_lds(1)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_bias_dropout_residual_ln_nodrop(cuda):
    from hetseq_amd.ops.bert_ops import bias_dropout_residual_ln

    torch.manual_seed(1)
    T, H = 512, 768
    a = torch.randn(T, H, device=cuda, requires_grad=True)
    bias = torch.randn(H, device=cuda, requires_grad=True)
    r = torch.randn(T, H, device=cuda, requires_grad=True)
    g = torch.rand(H, device=cuda, requires_grad=True)
    be = torch.randn(H, device=cuda, requires_grad=True)
    y = bias_dropout_residual_ln(a, bias, r, g, be, p=0.0)
    leaves = [t.detach().clone().requires_grad_() for t in (a, bias, r, g, be)]
    y2 = _ref_ln(leaves[0] + leaves[1] + leaves[2], leaves[3], leaves[4])
    _close(y, y2, msg="bdrln fwd")
    dy = torch.randn_like(y)
    y.backward(dy)
    y2.backward(dy)
    for t1, t2, n in zip((a, bias, r, g, be), leaves, "a bias r g b".split()):
        _close(t1.grad, t2.grad, 1e-4, 1e-3, "bdrln d" + n)


def test_bias_dropout_residual_ln_dropout_consistent(cuda):
    """With dropout, the backward must use exactly the forward's mask."""
    from hetseq_amd.ops.bert_ops import bias_dropout_residual_ln
    from hetseq_amd.runtime import rng

    torch.manual_seed(2)
    T, H, p = 256, 768, 0.1
    a = torch.randn(T, H, device=cuda, requires_grad=True)
    bias = torch.zeros(H, device=cuda)
    r = torch.zeros(T, H, device=cuda)
    g = torch.ones(H, device=cuda)
    be = torch.zeros(H, device=cuda)
    rng.set_seed(1234)
    y = bias_dropout_residual_ln(a, bias, r, g, be, p=p)
    # recover the mask through the gradient of sum(y * w) with LN folded out: use identity check instead
    rng.set_seed(1234)
    y_again = bias_dropout_residual_ln(a.detach(), bias, r, g, be, p=p)
    assert torch.equal(y.detach(), y_again), "Philox mask not reproducible for a fixed (seed, offset)"
    # kept fraction ~ 1-p: a zero row element of dropout output shows up as pre-LN zero; check via z
    from hetseq_amd.ops import bert_ops

    rng.set_seed(99)
    _, z, _, _ = bert_ops.ln_fwd(torch.ones(T, H, device=cuda), g, be, bias=bias, resid=r, p=p, mode=1,
                                 seed=99, off=0)
    kept = (z != 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.01, kept
    assert torch.allclose(z[z != 0], torch.full_like(z[z != 0], 1 / (1 - p)))
    # gradient check against an explicit-mask reference at the same (seed=99, off=0) site
    mask = (z != 0).float() / (1 - p)
    a2 = a.detach().clone().requires_grad_()
    y2 = _ref_ln(a2 * mask, g, be)
    y_f, z_f, m_f, rs_f = bert_ops.ln_fwd(a2.detach(), g, be, bias=bias, resid=r, p=p, mode=1, seed=99, off=0)
    _close(y_f, y2.detach(), msg="masked fwd")
    dy = torch.randn_like(y_f)
    y2.backward(dy)
    dz, da, dg, db, dbias = bert_ops.ln_bwd(dy, z_f, m_f, rs_f, g, p, 1, 99, 0, True, True)
    _close(da, a2.grad, 1e-4, 1e-4, "dropout-masked grad")


def test_bias_gelu(cuda):
    from hetseq_amd.models.bert import bias_gelu as ref
    from hetseq_amd.ops.bert_ops import bias_gelu

    torch.manual_seed(3)
    x = torch.randn(1000, 3072, device=cuda, requires_grad=True)
    b = torch.randn(3072, device=cuda, requires_grad=True)
    y = bias_gelu(x, b)
    x2, b2 = x.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    y2 = ref(b2, x2)
    _close(y, y2, 1e-5, 1e-5, "gelu fwd")
    dy = torch.randn_like(y)
    y.backward(dy)
    y2.backward(dy)
    _close(x.grad, x2.grad, 1e-4, 1e-5, "gelu dx")
    _close(b.grad, b2.grad, 1e-4, 1e-3, "gelu db")


def _ref_attention(qkv, mask, B, S, NH):
    H = qkv.shape[1] // 3
    q, k, v = qkv.view(B, S, 3, NH, 64).permute(2, 0, 3, 1, 4)
    scores = torch.matmul(q, k.transpose(-1, -2)) / 8.0
    scores = scores + ((1.0 - mask.float()) * -10000.0)[:, None, None, :]
    p = torch.softmax(scores, -1)
    return torch.matmul(p, v).permute(0, 2, 1, 3).reshape(B * S, H)


@pytest.mark.parametrize("B,S,NH", [(2, 128, 12), (3, 64, 4), (1, 512, 2), (2, 96, 2)])
def test_attention_fwd_bwd(cuda, B, S, NH):
    from hetseq_amd.ops.bert_ops import attention

    torch.manual_seed(4)
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda, requires_grad=True)
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[0, S - 17:] = 0
    if B > 1:
        mask[1, 5:9] = 0
    out = attention(qkv, mask, B, S, NH, 0.0)
    qkv2 = qkv.detach().clone().requires_grad_()
    out2 = _ref_attention(qkv2, mask, B, S, NH)
    _close(out, out2, 1e-4, 1e-5, "attn fwd")
    dout = torch.randn_like(out)
    out.backward(dout)
    out2.backward(dout)
    _close(qkv.grad, qkv2.grad, 1e-4, 1e-5, "attn dqkv")


def _keep_mask(dmask, BH, S):
    """[BH, S(query), S(key)] float keep mask unpacked from the forward's packed keep bits."""
    w = dmask.view(BH, S, S // 32, 1)
    sh = torch.arange(32, device=dmask.device, dtype=torch.int32)
    return ((w >> sh) & 1).reshape(BH, S, S).double()


def _ref_attention_drop(qkv, mask, B, S, NH, keep, p):
    H = qkv.shape[1] // 3
    q, k, v = qkv.view(B, S, 3, NH, 64).permute(2, 0, 3, 1, 4)
    scores = torch.matmul(q, k.transpose(-1, -2)) / 8.0
    scores = scores + ((1.0 - mask.to(qkv.dtype)) * -10000.0)[:, None, None, :]
    prob = torch.softmax(scores, -1)
    if p > 0:
        thr = min(65536, int(p * 65536.0 + 0.5))
        prob = prob * keep.view(B, NH, S, S) * (65536.0 / (65536 - thr))
    return torch.matmul(prob, v).permute(0, 2, 1, 3).reshape(B * S, H)


@pytest.mark.parametrize("S", [256, 384, 512])
@pytest.mark.parametrize("B,NH", [(1, 2), (8, 12)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_long_seq_fwd_bwd_vs_fp64(cuda, S, B, NH, p):
    """Phase-2 lengths (S > 128: chunked forward, two-kernel backward) against an fp64 autograd
    reference that applies the forward's own keep bits (regression grid of the round-1 fault)."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(40 + S + B)
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda)
    bias = torch.randn(3 * H, device=cuda) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[0, S - 37:] = 0
    if B > 1:
        mask[B - 1, 3:11] = 0
    out, (lse, dmask) = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 17, 5, bias=bias)
    dout = torch.randn_like(out)
    dqkv = bert_ops.attn_bwd(qkv, mask, out, dout, (lse, dmask), B, S, NH, p, bias=bias)
    torch.cuda.synchronize()
    keep = _keep_mask(dmask, B * NH, S) if p > 0 else None
    x = (qkv.double() + bias.double()).requires_grad_()
    ref = _ref_attention_drop(x, mask, B, S, NH, keep, p)
    ref.backward(dout.double())
    _close(out, ref, 1e-4, 1e-6, "long-seq attn fwd")
    _close(dqkv, x.grad, 1e-4, 1e-6, "long-seq attn dqkv")


@pytest.mark.parametrize("B,S,NH,p", [(2, 128, 12, 0.0), (2, 96, 2, 0.1), (1, 512, 2, 0.0), (2, 192, 2, 0.1),
                                       (3, 64, 4, 0.1), (2, 256, 12, 0.0), (8, 512, 12, 0.1), (1, 288, 2, 0.1)])
@pytest.mark.parametrize("data", ["uniform", "wide"])
def test_attention_h3_matches_fp64(cuda, B, S, NH, p, data):
    """fp32 attention on three split-fp16 products with in-kernel power-of-two scales (attention_h3.hip,
    the default fp32 engine): forward and backward against the exact-fp32 MFMA kernels on the same
    forward (same keep bits), and against fp64 autograd at the exact-fp32 kernels' error level.
    'wide': V and dO token magnitudes spread over three decades inside every head (and 100x outlier
    V rows), Q / K over one decade (scores stay O(10), as from LayerNorm'd inputs: a saturated softmax
    only measures the score rounding of either engine), so the chunk scales, the accumulator
    rescaling between chunks and the running dS exponent are exercised."""
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops._C import hip

    torch.manual_seed(70 + S + B)
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda)
    if data == "wide":
        qkv[:, :2 * H] *= torch.pow(10.0, torch.empty(B * S, 1, device=cuda).uniform_(-0.5, 0.5))
        qkv[:, 2 * H:] *= torch.pow(10.0, torch.empty(B * S, 1, device=cuda).uniform_(-1.5, 1.5))
        qkv[::37, 2 * H:] *= 100.0
    bias = torch.randn(3 * H, device=cuda) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[-1, S // 3:] = 0
    old = hip().attn_fp32_mode()
    try:
        hip().set_attn_fp32_mode(0)
        out32, saved32 = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 3, 11, bias=bias)
        hip().set_attn_fp32_mode(2)
        out3, saved3 = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 3, 11, bias=bias)
        dout = torch.randn_like(out32)
        if data == "wide":
            dout *= torch.pow(10.0, torch.empty(B * S, 1, device=cuda).uniform_(-1.5, 1.5))
        g3 = bert_ops.attn_bwd(qkv, mask, out32, dout, saved32, B, S, NH, p, bias=bias)
        # the same backward with dQ from the stored dS (the layer program's path)
        from hetseq_amd.ops import h3p
        g3ds = bert_ops.attn_bwd_h3p(qkv, mask, out32, dout, saved32, B, S, NH, p, bias,
                                     h3p.empty(B * S, 3 * H, cuda), fp32=True, ds=True)
        hip().set_attn_fp32_mode(0)
        g32 = bert_ops.attn_bwd(qkv, mask, out32, dout, saved32, B, S, NH, p, bias=bias)
    finally:
        hip().set_attn_fp32_mode(old)
    torch.cuda.synchronize()
    if p > 0:
        assert torch.equal(saved3[1], saved32[1])
    keep = _keep_mask(saved32[1], B * NH, S) if p > 0 else None
    x = (qkv.double() + bias.double()).requires_grad_()
    ref = _ref_attention_drop(x, mask, B, S, NH, keep, p)
    ref.backward(dout.double())
    # 22-bit operands against fp32's 24: where a few terms dominate a short contraction (the wide data,
    # 128 queries) the representation error shows, up to 4x the exact-fp32 kernels'; on uniform data the
    # accumulation rounding of both dominates (within 2x)
    f = 2.0 if data == "uniform" else 4.0
    e3 = float((out3.double() - ref.detach()).abs().max())
    e32 = float((out32.double() - ref.detach()).abs().max())
    assert e3 <= f * e32 + 1e-7, ("forward", e3, e32)
    g3e = float((g3.double() - x.grad).abs().max())
    g32e = float((g32.double() - x.grad).abs().max())
    assert g3e <= f * g32e + 1e-7, ("backward", g3e, g32e)
    assert torch.isfinite(g3).all()
    gdse = float((g3ds.double() - x.grad).abs().max())
    assert gdse <= f * g32e + 1e-7, ("backward, dQ from the stored dS", gdse, g32e)
    H3 = 3 * H  # the K / V gradients are the same kernel's either way
    assert torch.equal(g3ds.view(-1, H3)[:, H:], g3.view(-1, H3)[:, H:])


@pytest.mark.parametrize("S,engine", [(128, 2), (512, 2), (128, 0)])
def test_attention_writes_output_amax(cuda, S, engine):
    """The |max| slot the attention launch fills for the h3 GEMMs (ctx forward, dqkv backward): written by
    the h3 kernels themselves, by a separate pass for the other engines -- exactly max |output| either way."""
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops._C import hip

    torch.manual_seed(5 + S)
    B, NH = 4, 12
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda)
    bias = torch.randn(3 * H, device=cuda) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[-1, S // 2:] = 0
    sf = torch.zeros(G.SLOT_FLOATS, device=cuda)
    sb = torch.zeros(G.SLOT_FLOATS, device=cuda)
    old = hip().attn_fp32_mode()
    try:
        hip().set_attn_fp32_mode(engine)
        ctx, saved = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 3, 11, bias=bias, amax=sf)
        dctx = torch.randn_like(ctx)
        dqkv = bert_ops.attn_bwd(qkv, mask, ctx, dctx, saved, B, S, NH, 0.1, bias=bias, amax=sb)
    finally:
        hip().set_attn_fp32_mode(old)
    torch.cuda.synchronize()
    assert float(G.amax_value(sf)[0]) == float(ctx.abs().max())
    assert float(G.amax_value(sb)[0]) == float(dqkv.abs().max())


@pytest.mark.parametrize("n,bound", [(4096, 30522), (1, 5), (777, 2), (16384, 30522), (5000, 100000)])
def test_sort_keys_matches_stable_sort(cuda, n, bound):
    """The one-block LDS key sort returns torch.sort(stable=True)'s keys and indices exactly."""
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops._C import hip

    torch.manual_seed(n)
    keys = torch.randint(0, bound, (n,), device=cuda, dtype=torch.int64)
    ok = torch.empty_like(keys)
    oo = torch.empty_like(keys)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    served = hip().sort_keys(keys.data_ptr(), n, bound, ok.data_ptr(), oo.data_ptr(), err.data_ptr(), 0) == 0
    assert served == (n <= 16384 and (n - 1).bit_length() + (bound - 1).bit_length() <= 32)
    k, o = bert_ops.sort_keys(keys, bound)
    rk, ro = torch.sort(keys, stable=True)
    assert torch.equal(k, rk) and torch.equal(o, ro)
    assert int(err.item()) == 0


def test_sort_keys_flags_out_of_range_keys(cuda):
    """A key outside [0, bound) no longer wraps silently: bit 2 of the error word is set (raised
    by check_device_errors) and the key sorts as clamped, so the output stays a permutation."""
    from hetseq_amd.ops._C import hip

    keys = torch.tensor([3, -1, 7, 2, 9, 0], device=cuda, dtype=torch.int64)
    ok, oo = torch.empty_like(keys), torch.empty_like(keys)
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    assert hip().sort_keys(keys.data_ptr(), 6, 8, ok.data_ptr(), oo.data_ptr(), err.data_ptr(), 0) == 0
    assert int(err.item()) & 4
    assert sorted(oo.tolist()) == list(range(6))
    assert ok.tolist() == [0, 0, 2, 3, 7, 7]


@pytest.mark.parametrize("B,S,NH", [(2, 128, 12), (2, 96, 2), (1, 512, 2)])
def test_attention_fwd_bf16_mfma(cuda, B, S, NH, monkeypatch):
    """bf16 matrix-core forward vs an fp64 reference on the same bf16 inputs (+ bias), and vs the fp32-MFMA path."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(21)
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda).bfloat16()
    bias = torch.randn(3 * H, device=cuda) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[-1, S // 3:] = 0
    out, (lse, _) = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.0, 0, 0, bias=bias)
    ref = _ref_attention((qkv.double() + bias.double()), mask, B, S, NH)
    _close(out, ref, 2e-2, 2e-2, "bf16 mfma attention fwd")
    monkeypatch.setenv("HETSEQ_ATTN_BF16_MFMA", "0")
    out32, (lse32, _) = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.0, 0, 0, bias=bias)
    _close(out, out32, 2e-2, 2e-2, "bf16 mfma vs fp32-mfma path")
    _close(lse, lse32, 1e-2, 2e-2, "lse")


@pytest.mark.parametrize("S,p", [(128, 0.0), (128, 0.1), (96, 0.1), (32, 0.0)])
def test_attention_bwd_bf16_mfma(cuda, S, p, monkeypatch):
    """bf16 matrix-core fused backward vs the fp32-MFMA fused backward on the same bf16 inputs."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(23)
    B, NH = 2, 4
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda).bfloat16()
    bias = torch.randn(3 * H, device=cuda) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[1, S // 2:] = 0
    out, lse = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 5, 7, bias=bias)
    dout = torch.randn_like(out)
    g16 = bert_ops.attn_bwd(qkv, mask, out, dout, lse, B, S, NH, p, bias=bias)
    monkeypatch.setenv("HETSEQ_ATTN_BF16_MFMA", "0")
    g32 = bert_ops.attn_bwd(qkv, mask, out, dout, lse, B, S, NH, p, bias=bias)
    _close(g16, g32, 3e-2, 3e-2, "bf16 mfma attention backward")
    if p == 0.0:  # and against fp64 autograd on the bf16 inputs
        x = (qkv.double() + bias.double()).requires_grad_()
        _ref_attention(x, mask, B, S, NH).backward(dout.double())
        _close(g16, x.grad, 3e-2, 3e-2, "bf16 mfma attention backward vs fp64")


def test_attention_bf16_mfma_dropout_bits_match(cuda, monkeypatch):
    """The bf16 forward draws the same keep bits as the fp32 forward (shared Philox stream)."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(22)
    B, S, NH = 2, 128, 4
    qkv = torch.randn(B * S, 3 * NH * 64, device=cuda).bfloat16()
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    _, (_, bits) = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 9, 4)
    monkeypatch.setenv("HETSEQ_ATTN_BF16_MFMA", "0")
    _, (_, bits32) = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.1, 9, 4)
    assert torch.equal(bits, bits32)


@pytest.mark.parametrize("S", [32, 96, 128])
def test_attention_bwd_fused_matches_split(cuda, S, monkeypatch):
    """The one-block-per-head fused backward (S <= 128) equals the two-kernel path, with dropout + bias."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(12)
    B, NH, p = 2, 3, 0.1
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda)
    bias = torch.randn(3 * H, device=cuda) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[1, S // 2:] = 0
    out, lse = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 5, 7, bias=bias)
    dout = torch.randn_like(out)
    g_fused = bert_ops.attn_bwd(qkv, mask, out, dout, lse, B, S, NH, p, bias=bias)
    monkeypatch.setenv("HETSEQ_ATTN_BWD", "split")
    g_split = bert_ops.attn_bwd(qkv, mask, out, dout, lse, B, S, NH, p, bias=bias)
    _close(g_fused, g_split, 1e-5, 1e-6, "fused vs split attention backward")


def test_attention_fully_masked_row(cuda):
    """-10000 additive mask (not -inf): a fully masked sequence still attends (Q27)."""
    from hetseq_amd.ops.bert_ops import attention

    torch.manual_seed(5)
    B, S, NH = 1, 64, 2
    qkv = torch.randn(B * S, 3 * NH * 64, device=cuda)
    mask = torch.zeros(B, S, dtype=torch.int64, device=cuda)
    out = attention(qkv, mask, B, S, NH, 0.0)
    # every score sits near -10000, where fp32 resolves 2^-10: the fp32 reference itself is off the exact
    # result by ~1e-4 there, so the kernel is held to the fp64 result within twice the fp32 reference's
    # own error (the h3 softmax runs in base 2 and rounds differently from the natural-base reference)
    ref64 = _ref_attention(qkv.double(), mask, B, S, NH)
    e32 = (_ref_attention(qkv, mask, B, S, NH).double() - ref64).abs().max().item()
    err = (out.double() - ref64).abs().max().item()
    assert err <= 2 * e32 + 1e-5, "masked fwd: max err %.3e vs the fp32 reference's %.3e" % (err, e32)
    assert torch.isfinite(out).all()


def test_attention_dropout(cuda):
    """Dropout: deterministic for a fixed seed, unbiased, and backward consistent with forward."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(6)
    B, S, NH, p = 2, 128, 4, 0.1
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda)
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    o1, l1 = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 7, 0)
    o2, l2 = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 7, 0)
    assert torch.equal(o1, o2)
    o3, _ = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 8, 0)
    assert not torch.equal(o1, o3)
    # expectation over many seeds approaches the no-dropout output
    acc = torch.zeros_like(o1)
    n = 64
    for s in range(n):
        acc += bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 1000 + s, 0)[0]
    ref, _ = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.0, 0, 0)
    assert (acc / n - ref).abs().mean().item() < 0.05 * ref.abs().mean().item() + 1e-3
    # gradient consistency: finite-difference of sum(out * w) along a random direction
    qkv64 = qkv.double()
    w = torch.randn_like(o1)
    dqkv = bert_ops.attn_bwd(qkv, mask, o1, w, l1, B, S, NH, p, 7, 0)
    d = torch.randn_like(qkv) * 1e-2
    fp = (bert_ops.attn_fwd(qkv + d, mask, B, S, NH, p, 7, 0)[0] * w).sum().item()
    fm = (bert_ops.attn_fwd(qkv - d, mask, B, S, NH, p, 7, 0)[0] * w).sum().item()
    fd = (fp - fm) / 2
    an = (dqkv * d).sum().item()
    assert abs(fd - an) <= 2e-2 * abs(an) + 1e-3, (fd, an)


def test_embedding_fwd_bwd(cuda):
    from hetseq_amd.ops.bert_ops import FusedEmbedding

    torch.manual_seed(7)
    B, S, V, H, P, TV = 4, 128, 1000, 768, 512, 2
    ids = torch.randint(0, V, (B, S), device=cuda)
    tt = torch.randint(0, TV, (B, S), device=cuda)
    ww = torch.randn(V, H, device=cuda, requires_grad=True)
    wp = torch.randn(P, H, device=cuda, requires_grad=True)
    wt = torch.randn(TV, H, device=cuda, requires_grad=True)
    g = torch.rand(H, device=cuda, requires_grad=True)
    b = torch.randn(H, device=cuda, requires_grad=True)
    y = FusedEmbedding.apply(ids, tt, ww, wp, wt, g, b, 0.0, 1e-12, torch.float32)
    leaves = [t.detach().clone().requires_grad_() for t in (ww, wp, wt, g, b)]
    pos = torch.arange(S, device=cuda).expand(B, S)
    e = F.embedding(ids, leaves[0]) + F.embedding(pos, leaves[1]) + F.embedding(tt, leaves[2])
    y2 = _ref_ln(e, leaves[3], leaves[4]).view(B * S, H)
    _close(y, y2, 1e-4, 1e-5, "emb fwd")
    dy = torch.randn_like(y)
    y.backward(dy)
    y2.backward(dy)
    for t1, t2, n in zip((ww, wp, wt, g, b), leaves, ["word", "pos", "type", "gamma", "beta"]):
        _close(t1.grad, t2.grad, 1e-4, 1e-3, "emb d" + n)


def test_embedding_backward_bitwise_deterministic(cuda):
    """Sorted-run scatter (no atomics): repeated ids give bitwise-identical gradients run to run."""
    from hetseq_amd.ops.bert_ops import FusedEmbedding

    torch.manual_seed(8)
    B, S, V, H = 8, 128, 50, 768  # 50-word vocab: every id repeats ~20 times
    ids = torch.randint(0, V, (B, S), device=cuda)
    tt = torch.randint(0, 2, (B, S), device=cuda)
    dy = torch.randn(B * S, H, device=cuda)
    from hetseq_amd.runtime import rng

    grads = []
    for _ in range(3):
        rng.set_seed(123)  # same dropout stream every repetition
        ws = [torch.randn(n, H, device=cuda, generator=torch.Generator(cuda).manual_seed(1)).requires_grad_()
              for n in (V, 512, 2)]
        g = torch.ones(H, device=cuda, requires_grad=True)
        b = torch.zeros(H, device=cuda, requires_grad=True)
        FusedEmbedding.apply(ids, tt, ws[0], ws[1], ws[2], g, b, 0.1, 1e-12, torch.float32).backward(dy)
        grads.append([w.grad.clone() for w in ws])
    for other in grads[1:]:
        for a, c in zip(grads[0], other):
            assert torch.equal(a, c)


@pytest.mark.parametrize("rows,N", [(640, 768), (257, 3072), (96, 1000)])
def test_gelu_bwd_colsum_reports_amax(cuda, rows, N):
    """The GELU backward + column-sum kernel maxes |dx| into a given slot (the MLM transform's h3
    operand scale); dx and the column sums are unchanged by it."""
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops.bert_ops import gelu_bwd_colsum

    gen = torch.Generator(device=cuda).manual_seed(6)
    dy, x = (torch.randn(rows, N, device=cuda, generator=gen) for _ in range(2))
    b = torch.randn(N, device=cuda, generator=gen)
    slot = torch.zeros(G.SLOT_FLOATS, device=cuda)
    dx1, db1 = gelu_bwd_colsum(dy, x, b, amax=slot)
    dx0, db0 = gelu_bwd_colsum(dy, x, b)
    assert torch.equal(dx1, dx0) and torch.equal(db1, db0)
    assert G.amax_value(slot).max().item() == dx0.abs().max().item()


@pytest.mark.parametrize("V,ld", [(30522, 30720), (4099, 4104), (1024, 1024), (1025, 1028)])
def test_cross_entropy_aligned_rows(cuda, V, ld):
    """fp32 logits whose rows start 16-B aligned (the MLM decoder's padded buffer) take the float4
    kernels: loss, logsumexp and the in-place dlogits against PyTorch in fp64, a few rows shifted
    by +-40 (online max), the pad columns untouched."""
    from hetseq_amd.ops import bert_ops as B

    gen = torch.Generator(device=cuda).manual_seed(4)
    rows = 160
    buf = torch.randn(rows, ld, device=cuda, generator=gen)
    buf[::7] += 40.0
    buf[3::11] -= 40.0
    pad = buf[:, V:].clone()
    x = buf[:, :V]
    lab = torch.randint(0, V, (rows,), device=cuda, generator=gen)
    lab[::5] = -1
    xd = x.double().clone().requires_grad_()
    ref = F.cross_entropy(xd, lab, ignore_index=-1)
    ref.backward()
    stats, lse = B.xent_fwd(x, lab)  # stats = (mean loss, valid rows)
    _close(stats[0], ref, 1e-5, 1e-6, "xent fwd")
    _close(lse, torch.logsumexp(x.double(), 1), 1e-6, 1e-5, "lse")
    from hetseq_amd.ops import gemm as G

    slot = torch.zeros(G.SLOT_FLOATS, device=cuda)
    B.xent_bwd_(x, lab, lse, torch.ones(1, device=cuda), stats, amax=slot)
    _close(x, xd.grad, 1e-4, 1e-9, "xent bwd")
    assert torch.equal(buf[:, V:], pad)
    assert G.amax_value(slot).max().item() == x.abs().max().item()  # the written gradient's |max|


def test_cross_entropy(cuda):
    from hetseq_amd.ops.bert_ops import cross_entropy

    torch.manual_seed(8)
    for V in (2, 30522):
        x = torch.randn(200, V, device=cuda, requires_grad=True)
        lab = torch.randint(0, V, (200,), device=cuda)
        lab[::3] = -1
        l1 = cross_entropy(x, lab)
        x2 = x.detach().clone().requires_grad_()
        l2 = F.cross_entropy(x2, lab, ignore_index=-1)
        _close(l1, l2, 1e-5, 1e-6, "xent fwd")
        l1.backward()
        l2.backward()
        _close(x.grad, x2.grad, 1e-4, 1e-8, "xent bwd")


@pytest.mark.parametrize("engine,ksplit", [("native", 1), ("x6", 1), ("x6", 2), ("x6", 0), ("h3", 1), ("h3", 2),
                                           ("h3", 0)])
@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 128), (4096, 768, 768), (4096, 3072, 768), (768, 3072, 4096),
                                   (300, 130, 72), (640, 30522, 64)])
def test_gemm_hip(cuda, engine, ksplit, ta, tb, M, N, K):
    from hetseq_amd.models.bert import f_gelu
    from hetseq_amd.ops import gemm as G

    if engine == "native" and ksplit != 1:
        pytest.skip("split-K is a split-bf16 engine feature")

    torch.manual_seed(9)
    a = torch.randn((K, M) if ta else (M, K), device=cuda)
    b = torch.randn((N, K) if tb else (K, N), device=cuda)
    bias = torch.randn(N, device=cuda)
    ref = (a.t() if ta else a).double() @ (b.t() if tb else b).double()
    out = torch.full((M, N), float("nan"), device=cuda)
    kw = dict(fp32=engine, ksplit=ksplit)
    served = G._hip_gemm(a, b, ta, tb, out, **kw)
    if M % 64 or N % 64 or K % 32:
        assert not served and torch.isnan(out).all()  # unsupported shape: nothing launched
        return
    assert served
    torch.cuda.synchronize()
    _close(out, ref, 1e-5, 1e-4, "gemm")
    c0 = torch.randn(M, N, device=cuda)
    out.copy_(c0)
    assert G._hip_gemm(a, b, ta, tb, out, beta=1.0, **kw)
    _close(out, ref + c0.double(), 1e-5, 1e-4, "gemm beta")
    if (ta, tb) == (0, 1):
        assert G._hip_gemm(a, b, ta, tb, out, bias=bias, epi=G.EPI_BIAS, **kw)
        _close(out, ref + bias.double(), 1e-5, 1e-4, "gemm+bias")
        out.copy_(c0)
        assert G._hip_gemm(a, b, ta, tb, out, bias=bias, epi=G.EPI_BIAS, beta=1.0, **kw)
        _close(out, ref + bias.double() + c0.double(), 1e-5, 1e-4, "gemm+bias beta")
        aux = torch.empty_like(out)
        assert G._hip_gemm(a, b, ta, tb, out, bias=bias, epi=G.EPI_GELU, aux=aux, **kw)
        _close(aux, ref, 1e-5, 1e-4, "gemm gelu pre")
        _close(out, f_gelu(ref + bias.double()), 1e-5, 1e-4, "gemm gelu")
    if (ta, tb) == (0, 0):
        pre = torch.randn(M, N, device=cuda)
        part = torch.empty(((M + 63) // 64, N), device=cuda)
        db = torch.randn(N, device=cuda)
        db0 = db.clone()
        assert G._hip_gemm(a, b, ta, tb, out, bias=bias, epi=G.EPI_DGELU, aux=pre, part=part, colsum=db,
                           colsum_acc=True, **kw)
        x = (pre.double() + bias.double()).requires_grad_()
        f_gelu(x).backward(ref)
        _close(out, x.grad, 1e-5, 1e-4, "gemm dgelu")
        _close(db, db0.double() + x.grad.sum(0), 1e-5, 1e-3, "gemm dgelu colsum")


@pytest.mark.parametrize("engine", ["x6", "h3"])
def test_gemm_splitk_deterministic(cuda, engine):
    """Split-K partial slabs are summed in slice order by one reduction pass: repeated runs are
    bitwise identical."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(5)
    a = torch.randn(4096, 768, device=cuda)
    b = torch.randn(4096, 1024, device=cuda)
    first = torch.empty(768, 1024, device=cuda)
    assert G._hip_gemm(a, b, 1, 0, first, fp32=engine, ksplit=4)
    ref = a.double().t() @ b.double()
    _close(first, ref, 1e-5, 1e-4, "splitk")
    for _ in range(20):
        out = torch.empty_like(first)
        assert G._hip_gemm(a, b, 1, 0, out, fp32=engine, ksplit=4)
        assert torch.equal(out, first)


@pytest.mark.parametrize("engine", ["x6", "h3"])
@pytest.mark.parametrize("ta,tb,M,N,K,ks", [(1, 0, 768, 3072, 4096, 2), (1, 0, 768, 768, 4096, 4),
                                            (0, 1, 4096, 768, 3072, 2), (0, 0, 4096, 768, 768, 2),
                                            (1, 0, 256, 384, 1024, 8)])
def test_gemm_splitk_reduce_pass_and_colsum_fold(cuda, engine, ta, tb, M, N, K, ks):
    """Split-K finished by the fixed-order reduce pass -- plain, accumulating (beta 1), with a bias,
    with the weight gradient's column sums folded into that pass or summed by their own reduce_rows
    launch (bitwise the same) -- against fp64."""
    from hetseq_amd.ops import gemm as G

    gen = torch.Generator(device=cuda).manual_seed(21)
    a = torch.randn((K, M) if ta else (M, K), device=cuda, generator=gen)
    b = torch.randn((N, K) if tb else (K, N), device=cuda, generator=gen)
    bias = torch.randn(N, device=cuda, generator=gen)
    c0 = torch.randn(M, N, device=cuda, generator=gen)
    cs0 = torch.randn(M, device=cuda, generator=gen)

    def run(beta, with_bias, wcol):
        out = c0.clone()
        kw = dict(fp32=engine, ksplit=ks, beta=beta)
        if with_bias:
            kw.update(bias=bias, epi=G.EPI_BIAS)
        cs = None
        if wcol:
            cs = cs0.clone()
            kw.update(part=torch.empty((ks, M), device=cuda), colsum=cs, colsum_acc=beta != 0.0)
        assert G._hip_gemm(a, b, ta, tb, out, **kw)
        return out, cs

    ad, bd = (a.t() if ta else a).double(), (b.t() if tb else b).double()
    ref = ad @ bd
    cases = [(0.0, False, False), (1.0, False, False)]
    if (ta, tb) == (0, 1):
        cases.append((1.0, True, False))
    if ta:
        cases += [(1.0, False, True), (0.0, False, True)]
    try:
        for beta, with_bias, wcol in cases:
            o0, c0_ = run(beta, with_bias, wcol)
            want = ref + beta * c0.double() + (bias.double() if with_bias else 0.0)
            _close(o0, want, 1e-5, 1e-4, "splitk beta=%g bias=%d" % (beta, with_bias))
            if wcol:
                _close(c0_, ad.sum(1) + (cs0.double() if beta else 0.0), 1e-5, 1e-4, "splitk colsum")
                G.hip().set_wcol_fold(0)  # the bias gradient by its own reduce_rows pass
                o2, c2 = run(beta, with_bias, wcol)
                G.hip().set_wcol_fold(1)
                assert torch.equal(o2, o0) and torch.equal(c2, c0_)
    finally:
        G.hip().set_wcol_fold(1)


@pytest.mark.parametrize("engine", ["x6", "h3"])
def test_gemm_dgelu_without_colsum(cuda, engine):
    """The dGELU data-gradient epilogue with no column partials (the FFN-in bias gradient then comes
    from the weight-gradient launch) writes the same dpre, bitwise, as with them."""
    from hetseq_amd.ops import gemm as G

    gen = torch.Generator(device=cuda).manual_seed(3)
    T, N, K = 4096, 3072, 768
    dy = torch.randn(T, K, device=cuda, generator=gen)
    w = torch.randn(K, N, device=cuda, generator=gen) * 0.05
    pre = torch.randn(T, N, device=cuda, generator=gen)
    b = torch.randn(N, device=cuda, generator=gen)
    out1, out0 = torch.empty(T, N, device=cuda), torch.empty(T, N, device=cuda)
    db = torch.zeros(N, device=cuda)
    part = torch.empty((T // 64, N), device=cuda)
    assert G._hip_gemm(dy, w, 0, 0, out1, b, G.EPI_DGELU, aux=pre, part=part, colsum=db, fp32=engine)
    assert G._hip_gemm(dy, w, 0, 0, out0, b, G.EPI_DGELU, aux=pre, fp32=engine)
    assert torch.equal(out0, out1)
    _close(db, out1.double().sum(0), 1e-5, 1e-3, "dgelu colsum")


def _wide_range(shape, cuda, gen, decades):
    """Gradient-like data: N(0,1) values times 10^u, u uniform in [-decades, 0] per ROW (some rows
    ~10^-decades of the tensor's max) and a few 100x outliers."""
    x = torch.randn(shape, device=cuda, generator=gen)
    x *= torch.pow(10.0, -decades * torch.rand((shape[0], 1), device=cuda, generator=gen))
    idx = torch.randint(0, x.numel(), (8,), device=cuda, generator=gen)
    x.view(-1)[idx] *= 100.0
    return x


@pytest.mark.parametrize("data", ["uniform", "wide"])
@pytest.mark.parametrize("ta,tb,M,N,K", [(0, 1, 4096, 2304, 768), (0, 0, 4096, 768, 3072), (1, 0, 768, 3072, 4096),
                                         (0, 1, 512, 512, 64)])
def test_gemm_h3_error_matches_fp32(cuda, data, ta, tb, M, N, K):
    """Split-fp16 products with per-tensor power-of-two scales carry fp32-level error: within 2x of
    the exact-fp32 MFMA kernel and of the library SGEMM against fp64 (units of |A|@|B|), on uniform
    data and on gradient-like data with 2^20 of dynamic range inside each tensor (rows scaled by
    10^-4..1, 100x outliers; operand magnitudes far from 1, so the scale must adapt) -- and NaN / inf
    in an operand propagate.  (The engine's window: elements down to 2^-18 of their tensor's |max|
    keep all 22 bits; test_gemm_h3_beyond_window measures the graceful loss below it.)"""
    from hetseq_amd.ops import gemm as G

    g = torch.Generator(device=cuda)
    g.manual_seed(21)
    if data == "uniform":
        a = torch.rand((K, M) if ta else (M, K), device=cuda, generator=g) * 2 - 1
        b = torch.rand((N, K) if tb else (K, N), device=cuda, generator=g) * 2 - 1
    else:
        # K >= 512: 4 decades of row scales + outliers (~2^22 of range: the dot products' fp32
        # rounding covers the bits the smallest rows lose); K = 64 (a head-sized product, little
        # accumulation to hide behind): 2 decades, inside the 2^18 window
        dec = 4.0 if K >= 512 else 2.0
        a = _wide_range((K, M) if ta else (M, K), cuda, g, dec) * 1e-5
        b = _wide_range((N, K) if tb else (K, N), cuda, g, dec) * 1e3
    At, Bt = (a.t() if ta else a), (b.t() if tb else b)
    ref = At.double() @ Bt.double()
    mag = At.double().abs() @ Bt.double().abs()
    out = torch.empty(M, N, device=cuda)

    def err():
        return float(((out.double() - ref).abs() / mag).max())

    errs = {}
    torch.mm(At, Bt, out=out)
    errs["blas"] = err()
    for eng in ("native", "x6", "h3"):
        assert G._hip_gemm(a, b, ta, tb, out, fp32=eng)
        errs[eng] = err()
    assert errs["h3"] <= 2.0 * max(errs["native"], errs["blas"]), errs
    # NaN / inf in an operand reach the product (never scaled away)
    a2 = a.clone()
    a2.view(-1)[17] = float("nan")
    assert G._hip_gemm(a2, b, ta, tb, out, fp32="h3")
    assert torch.isnan(out).any()
    a2.view(-1)[17] = float("inf")
    assert G._hip_gemm(a2, b, ta, tb, out, fp32="h3")
    assert (~torch.isfinite(out)).any()


def test_gemm_h3_beyond_window(cuda):
    """Rows 10^-6 below the tensor's |max| (beyond the h3 engine's 2^18 window): those rows lose
    bits gradually (their fp16 low terms go subnormal) -- measured here so the limit is explicit:
    the error stays bounded (under 1e-4 of |A|@|B|, against ~7e-7 for exact fp32) where the six-term
    bf16 split (x6) keeps fp32-level error at any range (HETSEQ_FP32_GEMM=x6 for such data)."""
    from hetseq_amd.ops import gemm as G

    g = torch.Generator(device=cuda)
    g.manual_seed(22)
    a = _wide_range((1024, 768), cuda, g, 6.0)
    b = torch.randn((768, 768), device=cuda, generator=g) * 0.02
    ref = a.double() @ b.double().t()
    mag = a.double().abs() @ b.double().abs().t()
    out = torch.empty(1024, 768, device=cuda)
    errs = {}
    for eng in ("x6", "h3"):
        assert G._hip_gemm(a, b, 0, 1, out, fp32=eng)
        errs[eng] = float(((out.double() - ref).abs() / mag).max())
    assert errs["x6"] < 1e-6 and errs["h3"] < 1e-4, errs


def test_amax_kernels(cuda):
    """|max| kernels: standalone (with NaN above inf) and the per-segment flat-buffer form."""
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops._C import hip, stream_handle

    x = torch.randn(1000, 36, device=cuda)
    x[3, 5] = -77.0
    assert G.amax_value(G.amax_of(x)).item() == 77.0
    big = torch.randn(1 << 22, device=cuda)  # many blocks: the slot's shards combine to the exact max
    big[123457] = 1234.5
    assert G.amax_value(G.amax_of(big)).item() == 1234.5
    x[7, 7] = float("inf")
    assert G.amax_value(G.amax_of(x)).item() == float("inf")
    x[9, 9] = float("nan")
    assert torch.isnan(G.amax_value(G.amax_of(x))).all()
    flat = torch.randn(4096, device=cuda)
    segs = [(0, 0, 100), (1, 100, 700), (0, 700, 1024)]  # (segment, first float4, end float4)
    tab = torch.tensor(segs, dtype=torch.int64, device=cuda)
    out = torch.zeros(2 * G.SLOT_FLOATS, device=cuda)
    hip().amax_seg(flat.data_ptr(), tab.data_ptr(), len(segs), out.data_ptr(), stream_handle())
    v = flat.view(-1, 4)
    want0 = torch.cat([v[0:100], v[700:1024]]).abs().max()
    got = G.amax_value(out)
    assert got[0].item() == want0.item() and got[1].item() == v[100:700].abs().max().item()


@pytest.mark.parametrize("ta,tb,M,N,K", [(0, 1, 4096, 2304, 768), (0, 0, 4096, 768, 3072), (1, 0, 768, 3072, 4096)])
def test_gemm_x6_error_matches_fp32(cuda, ta, tb, M, N, K):
    """Split-bf16 products carry fp32-level error: within 2x of the exact-fp32 MFMA kernel and of
    the library SGEMM, measured against fp64 in units of |A|@|B| (the scale a K-long fp32 dot
    product rounds on), and far below plain bf16."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(12)
    a = torch.rand((K, M) if ta else (M, K), device=cuda) * 2 - 1
    b = torch.rand((N, K) if tb else (K, N), device=cuda) * 2 - 1
    At, Bt = (a.t() if ta else a), (b.t() if tb else b)
    ref = At.double() @ Bt.double()
    mag = At.double().abs() @ Bt.double().abs()
    out = torch.empty(M, N, device=cuda)

    def err():
        return float(((out.double() - ref).abs() / mag).max())

    errs = {}
    torch.mm(At, Bt, out=out)
    errs["blas"] = err()
    for eng in ("native", "x6"):
        assert G._hip_gemm(a, b, ta, tb, out, fp32=eng)
        errs[eng] = err()
    out.copy_(At.bfloat16().float() @ Bt.bfloat16().float())
    errs["bf16"] = err()
    assert errs["x6"] <= 2.0 * max(errs["native"], errs["blas"]), errs
    assert errs["x6"] < 5e-7, errs
    assert errs["bf16"] > 100 * errs["x6"], errs


@pytest.mark.parametrize("mode", ["hip", "blas"])
def test_fused_ffn_gemms_dispatch(cuda, mode):
    """linear_gelu_fwd / linear_dgrad_dgelu give the same result on every engine."""
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops.bert_ops import bias_gelu_fwd, gelu_bwd_colsum

    torch.manual_seed(3)
    x = torch.randn(512, 256, device=cuda)
    w1 = torch.randn(1024, 256, device=cuda) * 0.05
    bi = torch.randn(1024, device=cuda) * 0.1
    dy = torch.randn(512, 256, device=cuda)
    w2 = torch.randn(256, 1024, device=cuda) * 0.05
    pre_ref = x @ w1.t()
    y_ref = bias_gelu_fwd(pre_ref, bi)
    dpre_ref, db_ref = gelu_bwd_colsum(dy @ w2, pre_ref, bi)
    old = G._MODE
    try:
        G.set_mode(mode)
        y, pre = G.linear_gelu_fwd(x, w1, bi)
        acc = torch.ones(1024, device=cuda)
        dpre, db = G.linear_dgrad_dgelu(dy, w2, pre, bi, db_acc=acc)
        assert db is acc
    finally:
        G.set_mode(old)
    _close(pre, pre_ref, 1e-5, 1e-4, "pre")
    _close(y, y_ref, 1e-5, 1e-4, "gelu")
    _close(dpre, dpre_ref, 1e-5, 1e-4, "dpre")
    _close(db, db_ref + 1.0, 1e-5, 1e-3, "db")


def test_bf16_wgrad_accumulates_fp32(cuda):
    """bf16 inputs, fp32 flat-grad output with beta=1 (library path, no temporary)."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(4)
    dy = torch.randn(256, 192, device=cuda).bfloat16()
    x = torch.randn(256, 128, device=cuda).bfloat16()
    g = torch.randn(192, 128, device=cuda)
    ref = g.double() + dy.double().t() @ x.double()
    G.linear_wgrad(dy, x, out=g, accumulate=True)
    _close(g, ref, 1e-5, 1e-3, "bf16 wgrad acc")
    G.linear_wgrad(dy, x, out=g, accumulate=False)
    _close(g, dy.double().t() @ x.double(), 1e-5, 1e-3, "bf16 wgrad")


def test_adam_flat_matches_reference(cuda):
    from argparse import Namespace

    from hetseq_amd.optim.optimizers import AdamReference, _Adam
    from hetseq_amd.runtime.flat import FlatParamStore

    torch.manual_seed(10)
    m = torch.nn.Sequential(torch.nn.Linear(64, 33), torch.nn.Linear(33, 7)).to(cuda)
    m_ref = torch.nn.Sequential(torch.nn.Linear(64, 33), torch.nn.Linear(33, 7)).to(cuda)
    m_ref.load_state_dict(m.state_dict())
    store = FlatParamStore(m)
    args = Namespace(lr=[1e-2], adam_betas="(0.9, 0.98)", adam_eps=1e-6, weight_decay=0.01)
    opt = _Adam(args, list(m.parameters()), store)
    ref = AdamReference(m_ref.parameters(), lr=1e-2, betas=(0.9, 0.98), eps=1e-6, weight_decay=0.01)
    for step in range(5):
        x = torch.randn(16, 64, device=cuda)
        opt.zero_grad()
        ref.zero_grad()
        m(x).pow(2).sum().backward()
        m_ref(x).pow(2).sum().backward()
        opt.multiply_grads(0.5)
        for p in m_ref.parameters():
            p.grad.mul_(0.5)
        n1 = opt.clip_grad_norm(1.0)
        n2 = torch.nn.utils.clip_grad_norm_(list(m_ref.parameters()), 1.0)
        _close(n1, n2, 1e-5, 1e-6, "grad norm")
        opt.step()
        ref.step()
    for p1, p2 in zip(m.parameters(), m_ref.parameters()):
        _close(p1, p2, 1e-5, 1e-6, "adam params")


def test_adadelta_flat_matches_torch(cuda):
    from argparse import Namespace

    from hetseq_amd.optim.optimizers import _Adadelta
    from hetseq_amd.runtime.flat import FlatParamStore

    torch.manual_seed(11)
    m = torch.nn.Linear(50, 20).to(cuda)
    m_ref = torch.nn.Linear(50, 20).to(cuda)
    m_ref.load_state_dict(m.state_dict())
    store = FlatParamStore(m)
    args = Namespace(lr=[1.0], adadelta_rho=0.9, adadelta_eps=1e-6, dadelta_weight_decay=0.001)
    opt = _Adadelta(args, list(m.parameters()), store)
    ref = torch.optim.Adadelta(m_ref.parameters(), lr=1.0, rho=0.9, eps=1e-6, weight_decay=0.001)
    for _ in range(4):
        x = torch.randn(8, 50, device=cuda)
        opt.zero_grad()
        ref.zero_grad()
        m(x).sum().backward()
        m_ref(x).sum().backward()
        opt.step()
        ref.step()
    for p1, p2 in zip(m.parameters(), m_ref.parameters()):
        _close(p1, p2, 1e-5, 1e-6, "adadelta")


def test_mlm_compact_and_gather(cuda):
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(12)
    T = 5000
    labels = torch.full((T,), -1, dtype=torch.int64, device=cuda)
    sel = torch.randperm(T, device=cuda)[:700].sort().values
    labels[sel] = torch.randint(0, 100, (700,), device=cuda)
    idx, lab, cnt = bert_ops.mlm_compact(labels, 800)
    assert int(cnt.item()) == 700
    assert torch.equal(idx[:700].long(), sel)
    assert torch.equal(lab[:700], labels[sel])
    assert (idx[700:] == -1).all() and (lab[700:] == -1).all()
    src = torch.randn(T, 256, device=cuda)
    g = bert_ops.gather_rows(src, idx)
    assert torch.equal(g[:700], src[sel]) and (g[700:] == 0).all()


@pytest.mark.parametrize("N", [3072, 30522, 2])
def test_colsum(cuda, N):
    from hetseq_amd.ops.bert_ops import colsum

    torch.manual_seed(13)
    x = torch.randn(700, N, device=cuda)
    _close(colsum(x), x.double().sum(0), 1e-5, 1e-4, "colsum")


@pytest.mark.parametrize("S", [128, 256])
def test_attention_folded_qkv_bias(cuda, S):
    """The QKV projection bias is added inside the attention kernels (fwd and both bwd kernels)."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(14)
    B, NH = 2, 3
    H = NH * 64
    qkv = torch.randn(B * S, 3 * H, device=cuda)
    bias = torch.randn(3 * H, device=cuda)
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[1, S - 20:] = 0
    out, aux = bert_ops.attn_fwd(qkv, mask, B, S, NH, 0.0, 0, 0, bias=bias)
    q2 = (qkv + bias).requires_grad_()
    ref = _ref_attention(q2, mask, B, S, NH)
    _close(out, ref, 1e-4, 1e-5, "biased attn fwd")
    dout = torch.randn_like(out)
    ref.backward(dout)
    dqkv = bert_ops.attn_bwd(qkv, mask, out, dout, aux, B, S, NH, 0.0, bias=bias)
    _close(dqkv, q2.grad, 1e-4, 1e-5, "biased attn dqkv")


def test_attention_dropout_bitmask_matches_philox(cuda):
    """Backward reads the forward's packed keep-bits; they must equal the Philox stream."""
    from hetseq_amd.ops import bert_ops

    torch.manual_seed(15)
    B, S, NH, p = 1, 64, 2, 0.25
    qkv = torch.randn(B * S, 3 * NH * 64, device=cuda)
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    _, (lse, dmask) = bert_ops.attn_fwd(qkv, mask, B, S, NH, p, 11, 3)
    words = dmask.view(B * NH, S, S // 32).cpu().numpy().astype("uint32")
    kept = sum(bin(int(w)).count("1") for w in words.ravel())
    frac = kept / float(B * NH * S * S)
    assert abs(frac - (1 - p)) < 0.02, frac
    # Dropout(p) on probabilities: with all-equal scores the output is mean(kept V) * 1/(1-p);
    # check one row against a host reconstruction from the bits
    qkv0 = qkv.clone()
    qkv0[:, : NH * 64] = 0  # Q = 0 -> uniform probabilities 1/S
    out, (_, dm0) = bert_ops.attn_fwd(qkv0, mask, B, S, NH, p, 11, 3)
    w = dm0.view(B * NH, S, S // 32)[0, 5].cpu().numpy().astype("uint32")
    keep = torch.tensor([(int(w[k // 32]) >> (k % 32)) & 1 for k in range(S)], dtype=torch.float32, device=cuda)
    v = qkv0[:, 2 * NH * 64: 2 * NH * 64 + 64]
    expect = (keep[:, None] * v).sum(0) / S / (1 - p)
    _close(out[5, :64], expect, 1e-4, 1e-5, "bitmask row")


def test_decoder_padded_vocab_products(cuda):
    """Tied-decoder products on the split-bf16 engine with a vocabulary that is not a multiple of
    the tile (padded to 128; missing weight rows / bias read as zero, gradient rows past V never
    written) against fp64, on the HIP engine explicitly."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(31)
    R, H, V = 256, 192, 1000
    t2 = torch.randn(R, H, device=cuda)
    w = torch.randn(V, H, device=cuda) * 0.05
    bias = torch.randn(V, device=cuda)
    old = G._MODE
    try:
        G.set_mode("hip")
        logits, buf = G.decoder_logits(t2, w, bias)
        assert buf is not None and buf.shape == (R, 1024) and logits.shape == (R, V)  # pad to 512
        ref = t2.double() @ w.double().t() + bias.double()
        _close(logits, ref, 1e-5, 1e-4, "decoder logits")
        assert torch.count_nonzero(buf[:, V:]) == 0
        buf[:, :V].copy_(torch.randn(R, V, device=cuda))  # stands in for dlogits (pad columns stay zero)
        dl = buf[:, :V].double()
        dt2 = G.decoder_dgrad(buf, w, V)
        _close(dt2, dl @ w.double(), 1e-5, 1e-4, "decoder dgrad")
        guard = torch.full((V + 64, H), 7.0, device=cuda)  # rows past V must stay untouched
        g0 = torch.randn(V, H, device=cuda)
        guard[:V].copy_(g0)
        G.decoder_wgrad(buf, t2, V, guard[:V], accumulate=True)
        _close(guard[:V], g0.double() + dl.t() @ t2.double(), 1e-5, 1e-4, "decoder wgrad")
        assert torch.all(guard[V:] == 7.0)
    finally:
        G.set_mode(old)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("acc", [False, True])
def test_pool_nsp_kernels_vs_fp64(cuda, dt, acc):
    """K08: pooler (first token, tanh) + NSP classifier + CE + the MLM-loss sum, fwd and bwd,
    against fp64 autograd (reference bert_modeling.py:506-516, 576-580, 883); labels of -1 are
    ignored; the input gradient is ADDED into the first-token rows of an existing dseq."""
    from hetseq_amd.ops._C import dtype_code, hip, stream_handle

    torch.manual_seed(50)
    B, S, H = 8, 32, 256
    seq = torch.randn(B * S, H, device=cuda).to(dt)
    Wp = torch.randn(H, H, device=cuda) * 0.05
    bp = torch.randn(H, device=cuda) * 0.1
    Wn = torch.randn(2, H, device=cuda) * 0.1
    bn = torch.randn(2, device=cuda) * 0.1
    lab = torch.tensor([0, 1, 1, -1, 0, 1, 0, 0], device=cuda)
    mlm = torch.tensor([1.5, 0.0], device=cuda)
    pooled = torch.empty(B, H, device=cuda)
    logits = torch.empty(B, 2, device=cuda)
    lse = torch.empty(B, device=cuda)
    stats = torch.empty(3, device=cuda)
    P = lambda t: t.data_ptr()  # noqa: E731
    hip().pool_nsp_fwd(dtype_code(seq), P(seq), B, S, H, P(Wp), P(bp), P(Wn), P(bn), P(lab), P(mlm), P(pooled),
                       P(logits), P(lse), P(stats), P(stats[2:]), stream_handle())
    x = seq.view(B, S, H)[:, 0].double().requires_grad_()
    leaves = [t.double().requires_grad_() for t in (Wp, bp, Wn, bn)]
    pr = torch.tanh(x @ leaves[0].t() + leaves[1])
    lg = pr @ leaves[2].t() + leaves[3]
    total = 1.5 + torch.nn.functional.cross_entropy(lg, lab, ignore_index=-1)
    _close(pooled, pr, 1e-5, 1e-6, "pooled")
    _close(logits, lg, 1e-5, 1e-6, "nsp logits")
    assert abs(stats[2].item() - total.item()) < 1e-5, (stats[2].item(), total.item())
    assert stats[0].item() == 7
    dl = torch.tensor([0.7], device=cuda)
    total.backward(torch.tensor(0.7, dtype=torch.float64, device=cuda))
    dseq = torch.randn(B * S, H, device=cuda).to(dt)
    dseq0 = dseq.clone()
    grads = [torch.randn_like(t) for t in (Wp, bp, Wn, bn)]
    base = [g.clone() for g in grads]
    dnsp = torch.empty(B, 2, device=cuda)
    dpre = torch.empty(B, H, device=cuda)
    part = torch.empty(B, 8, H, device=cuda)
    hip().pool_nsp_bwd(dtype_code(seq), P(dl), P(seq), P(dseq), B, S, H, P(Wp), P(Wn), P(lab), P(pooled), P(logits),
                       P(lse), P(stats), P(dnsp), P(dpre), P(part), P(grads[0]), P(grads[1]), P(grads[2]),
                       P(grads[3]), int(acc), stream_handle())
    old_first = dseq0.view(B, S, H)[:, 0].double()
    expect = old_first + x.grad
    # bf16 dseq: the sum is rounded once to bf16 (relative 2^-8 of its magnitude)
    atol = 1e-6 if dt == torch.float32 else 2.0 ** -8 * expect.abs().max().item()
    _close(dseq.view(B, S, H)[:, 0], expect, 1e-5, atol, "dx added into first-token rows")
    rest = dseq.view(B, S, H)[:, 1:]
    assert torch.equal(rest, dseq0.view(B, S, H)[:, 1:])
    for g, g0, leaf, n in zip(grads, base, leaves, ("dWp", "dbp", "dWn", "dbn")):
        expect = leaf.grad + (g0.double() if acc else 0)
        _close(g, expect, 1e-5, 1e-6, n)


def test_pretraining_heads_launch_no_torch_kernels(cuda):
    """The fused pre-training heads' NSP half is all hetseq kernels (no at::native launches)."""
    from torch.profiler import ProfilerActivity, profile

    from hetseq_amd.models.bert import BertConfig, BertForPreTraining

    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=512, hidden_size=256, num_hidden_layers=1,
                     num_attention_heads=4, intermediate_size=1024)
    model = BertForPreTraining(cfg).to(cuda).eval()
    model.max_predictions_per_seq = 4
    B, S = 4, 64
    ids = torch.randint(0, 512, (B, S), device=cuda)
    lab = torch.full((B, S), -1, dtype=torch.long, device=cuda)
    lab[:, 1:5] = ids[:, 1:5]
    nsp = torch.randint(0, 2, (B,), device=cuda)
    model(ids, torch.zeros_like(ids), torch.ones_like(ids), lab, nsp).backward()  # warm-up
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        model(ids, torch.zeros_like(ids), torch.ones_like(ids), lab, nsp).backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    if not names:
        pytest.skip("profiler recorded no device kernels on this build")
    assert any("pool_nsp" in n for n in names), names
    # the reference's pooler/NSP ops as torch kernels: bias+tanh, log-softmax / NLL (cross-entropy)
    bad = [n for n in names if "at::native" in n and any(k in n for k in ("tanh", "nll_loss", "log_softmax"))]
    assert not bad, bad


def _planes_operand(x, P):
    from hetseq_amd.ops import gemm as G

    assert P == 1  # (the split-bf16 P = 3 engine was retired for h3p)
    return G.Planes.of_bf16(x.bfloat16().contiguous())


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
@pytest.mark.parametrize("M,N,K,ks", [(256, 384, 512, 1), (640, 768, 768, 1), (384, 256, 1024, 4),
                                      (128, 128, 4096, 2)])
def test_gemm_planes_vs_fp64(cuda, ta, tb, M, N, K, ks, variant):
    """The bf16 plane engine in both layouts of each operand (k-contiguous b128 reads and
    mn-contiguous transposed reads) and with split-K, against fp64 of the bf16 operands: exact bf16
    products with fp32 accumulation."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(61 + M + N + K)
    a = torch.randn((K, M) if ta else (M, K), device=cuda)
    b = torch.randn((N, K) if tb else (K, N), device=cuda)
    pa, pb = _planes_operand(a, 1), _planes_operand(b, 1)
    out = torch.empty(M, N, device=cuda)
    assert G.gemm_planes(pa, pb, ta, tb, out, ksplit=ks, variant=variant)
    ad, bd = a.bfloat16().double(), b.bfloat16().double()
    ref = (ad.t() if ta else ad) @ (bd.t() if tb else bd)
    mag = (ad.abs().t() if ta else ad.abs()) @ (bd.abs().t() if tb else bd.abs())
    err = float(((out.double() - ref).abs() / mag).max())  # in units of |A|@|B|
    assert err < 1e-5, err


@pytest.mark.parametrize("ks", [1, 2])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_planes_valid_rows(cuda, ks, beta):
    """A padded weight-gradient product (the tied decoder over the padded vocabulary): M = 640 rows of
    which the first 555 are valid -- C has only those rows, nothing past them is read or written."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(67 + ks)
    R, Mp, Mv, N = 256, 640, 555, 256
    a = torch.randn(R, Mp, device=cuda)
    a[:, Mv:] = 0.0  # (the loss gradient's pad columns are zero)
    b = torch.randn(R, N, device=cuda)
    guard = torch.full((Mv + 8, N), 7.0, device=cuda)  # rows past Mv: a canary
    c0 = torch.randn(Mv, N, device=cuda)
    out = guard[:Mv]
    out.copy_(c0)
    assert G.gemm_planes(_planes_operand(a, 1), _planes_operand(b, 1), True, False, out, beta=beta, ksplit=ks,
                         mv=Mv)
    ad, bd = a.bfloat16().double(), b.bfloat16().double()
    ref = (ad.t() @ bd)[:Mv] + beta * c0.double()
    _close(out, ref, 1e-5, 1e-4, "planes valid rows")
    assert torch.equal(guard[Mv:], torch.full((8, N), 7.0, device=cuda))
    # not served: a bf16 C or a GELU epilogue with fewer valid rows
    assert not G.gemm_planes(_planes_operand(a, 1), _planes_operand(b, 1), True, False,
                             torch.empty(Mv, N, device=cuda, dtype=torch.bfloat16), mv=Mv)


@pytest.mark.parametrize("ks", [2, 4])
@pytest.mark.parametrize("epi_bias,beta", [(False, 0.0), (True, 0.0), (True, 1.0)])
def test_gemm_planes_bf16_splitk(cuda, ks, epi_bias, beta):
    """bf16 C through K slices: fp32 slabs summed in fixed order with the bias and beta applied
    once, rounded to bf16 at the end (the small-grid N = 768 products of the bf16 step)."""
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(63 + ks)
    T, K, N = 256, 1024, 384
    x, w = torch.randn(T, K, device=cuda).bfloat16(), (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    bias = torch.randn(N, device=cuda) if epi_bias else None
    c0 = torch.randn(T, N, device=cuda).bfloat16()
    y = c0.clone()
    ok = G.gemm_planes(G.Planes.of_bf16(x), G.Planes.of_bf16(w), False, True, y, bias,
                       G.EPI_BIAS if epi_bias else G.EPI_NONE, beta, ksplit=ks)
    assert ok
    ref = x.double() @ w.double().t() + (bias.double() if epi_bias else 0.0) + beta * c0.double()
    _close(y, ref, 1e-2, 1e-2, "bf16 split-K planes")


@pytest.mark.parametrize("P", [1])
def test_gemm_planes_epilogues(cuda, P):
    """bias, beta-accumulate, GELU (pre-activation kept) and dGELU + bias-gradient column sums."""
    from hetseq_amd.models.bert import f_gelu
    from hetseq_amd.ops import gemm as G

    torch.manual_seed(62)
    T, K, N = 256, 512, 384
    x, w, bias = torch.randn(T, K, device=cuda), torch.randn(N, K, device=cuda) * 0.05, torch.randn(N, device=cuda)
    px, pw = _planes_operand(x, P), _planes_operand(w, P)
    dt = torch.float32 if P == 3 else torch.bfloat16
    xd, wd = (x.double(), w.double()) if P == 3 else (x.bfloat16().double(), w.bfloat16().double())
    tol = 1e-5 if P == 3 else 1e-2
    # bias
    y = torch.empty(T, N, device=cuda, dtype=dt)
    assert G.gemm_planes(px, pw, False, True, y, bias, G.EPI_BIAS)
    _close(y, xd @ wd.t() + bias.double(), tol, tol, "planes bias")
    # beta accumulate (fp32 C)
    c0 = torch.randn(T, N, device=cuda)
    c = c0.clone()
    assert G.gemm_planes(px, pw, False, True, c, beta=1.0)
    _close(c, xd @ wd.t() + c0.double(), tol, tol, "planes beta")
    # GELU forward: y = gelu(pre + b), pre stored
    y, pre = G.linear_gelu_fwd(px, pw, bias)
    _close(pre, xd @ wd.t(), tol, tol, "planes gelu pre")
    _close(y, f_gelu(pre.double() + bias.double()), tol, tol, "planes gelu")
    # dGELU: dpre = (dy @ W) * gelu'(pre + b), db = colsum(dpre)
    dy = torch.randn(T, N, device=cuda)
    w2 = torch.randn(N, K, device=cuda) * 0.05  # dgrad operand [N][K]: dy[T,N] @ w2 -> [T, K]
    prek = torch.randn(T, K, device=cuda).to(dt)
    bk = torch.randn(K, device=cuda)
    dpre, db = G.linear_dgrad_dgelu(_planes_operand(dy, P), _planes_operand(w2, P), prek, bk)
    dyd, w2d = (dy.double(), w2.double()) if P == 3 else (dy.bfloat16().double(), w2.bfloat16().double())
    pk = prek.double().requires_grad_()
    f_gelu(pk + bk.double()).backward(dyd @ w2d)
    _close(dpre, pk.grad, tol, tol, "planes dgelu")
    _close(db, pk.grad.sum(0), tol, tol, "planes dgelu colsum")


def test_fast_stat_kernels_match_torch_ops(cuda):
    """stats_accum / stats_finalize (optim.hip) == the controller's torch-op bookkeeping, bit for bit."""
    import math

    from hetseq_amd.ops._C import hip, stream_handle

    st = torch.zeros(6, dtype=torch.float64, device=cuda)
    ref = torch.zeros(6, dtype=torch.float64, device=cuda)
    for i, (ss, ns, nt) in enumerate([(128, 32, 0), (128, 32, 7), (96, 24, 3)]):
        loss = torch.tensor(3.1 + i, dtype=torch.float32, device=cuda)
        nll = torch.tensor(2.7 - i, dtype=torch.float32, device=cuda)
        hip().stats_accum(st.data_ptr(), loss.data_ptr(), nll.data_ptr(), float(ss), float(ns), float(nt),
                          stream_handle())
        ref[0] += ss
        ref[1] += ns
        ref[2] += loss.double()
        ref[3] += nll.double()
        ref[4] += nt
    ln2 = math.log(2)
    scale = torch.empty(1, dtype=torch.float32, device=cuda)
    hip().stats_finalize(st.data_ptr(), ln2, 1.0, scale.data_ptr(), stream_handle())
    ref[2:4].div_(ref[0:1] * ln2)
    rs = torch.where(ref[0] > 0, 1.0 / ref[0].clamp(min=1e-30), torch.ones_like(ref[0])).float()
    torch.cuda.synchronize()
    assert torch.equal(st, ref), (st, ref)
    assert torch.equal(scale[0], rs), (scale, rs)
    z = torch.zeros(6, dtype=torch.float64, device=cuda)  # no samples: scale 1
    hip().stats_finalize(z.data_ptr(), ln2, 1.0, scale.data_ptr(), stream_handle())
    torch.cuda.synchronize()
    assert scale.item() == 1.0


def test_sumsq_segs_matches_fp64(cuda):
    """Sharded gradient norm (parallel/zero.py): one launch over a table of ranges -- aligned pieces,
    unaligned ends, ranges shorter than a float4 -- against the fp64 sums of squares."""
    from hetseq_amd.ops._C import hip, stream_handle

    torch.manual_seed(0)
    g = torch.randn(3_000_003, device=cuda) * torch.logspace(-3, 3, 3_000_003, device=cuda)
    segs = [(0, 65536), (70001, 70003), (100_000, 1_900_001), (1_900_005, 1_900_006), (2_000_001, 3_000_003)]
    rows, nb = [], 0
    for a, b in segs:
        rows += [a, b, nb]
        nb += max(1, min(hip().sumsq_blocks(), (b - a) // 16384))
    tab = torch.tensor(rows, dtype=torch.int64, device=cuda)
    p = torch.zeros(nb + 1, dtype=torch.float64, device=cuda)
    hip().sumsq_segs(g.data_ptr(), tab.data_ptr(), len(segs), nb, p.data_ptr(), stream_handle())
    hip().sum_partials(p.data_ptr(), nb, p[nb:].data_ptr(), stream_handle())
    ref = sum(float(g[a:b].double().pow(2).sum()) for a, b in segs)
    assert abs(float(p[nb]) - ref) <= 1e-6 * ref
