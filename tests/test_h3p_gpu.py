"""h3p: block-scaled split-fp16 operands and the GEMM over them (csrc/kernels/gemm_h3p.hip).

Numerics are measured against fp64 next to the exact-fp32 references (library SGEMM and the
exact-fp32 MFMA kernel), in units of |A| @ |B| -- the scale of an fp32 GEMM's own rounding."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _wide(shape, dev, gen, decades):
    """Gradient-like data: rows scaled over ``decades`` orders of magnitude, plus 100x outliers."""
    x = torch.randn(shape, device=dev, generator=gen)
    x *= torch.pow(10.0, -decades * torch.rand((shape[0], 1), device=dev, generator=gen))
    idx = torch.randint(0, x.numel(), (8,), device=dev, generator=gen)
    x.view(-1)[idx] *= 100.0
    return x


def _gelu_ref(x):  # the reference's erf-GELU constant (bert_modeling.py:104-111)
    return x * 0.5 * (1.0 + torch.erf(x / 1.41421))


def _gelu_grad_ref(x):
    c = 1.41421
    return 0.5 * (1.0 + torch.erf(x / c)) + x * (0.5641895835477563 / c) * torch.exp(-(x / c) ** 2)


def test_split_roundtrip_and_exponents(cuda):
    """Every element keeps 22 bits below its 32 x 32 block's |max| (block exponents, not one per
    tensor): blocks 2^40 apart in one matrix both round-trip to 2^-21 of their own |max|; zero and
    non-finite elements stay non-finite."""
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(1)
    x = torch.randn((256, 384), device=cuda, generator=g)
    x[:32, :32] *= 2.0 ** 40
    x[32:64, 64:96] *= 2.0 ** -40
    x[64:96, 96:128] = 0.0
    hp = h3p.split(x)
    y = hp.unsplit()
    xb = x.view(8, 32, 12, 32).abs().amax(dim=(1, 3))  # block |max|
    err = ((y - x).abs().view(8, 32, 12, 32).amax(dim=(1, 3)) / xb.clamp_min(1e-300))
    assert float(err[xb > 0].max()) <= 2.0 ** -21
    assert (y[64:96, 96:128] == 0).all()
    e = hp.exps.to(torch.int32)
    assert int(e[0, 0]) == 14 - int(torch.floor(torch.log2(xb[0, 0])).item())
    x2 = x.clone()
    x2[100, 200] = float("nan")
    x2[200, 300] = float("inf")
    y2 = h3p.split(x2).unsplit()
    # (an inf element's lo term is inf - inf: the pair reads back as NaN -- non-finite either way)
    assert torch.isnan(y2[100, 200]) and not torch.isfinite(y2[200, 300])


def test_blocked_layout_split_matches_row_major(cuda):
    """The blocked plane layout (32 x 32 blocks of 2 KB) holds bitwise the row-major planes' values,
    and a row window of it is a view of the same blocks."""
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(5)
    x = torch.randn((256, 384), device=cuda, generator=g) * torch.logspace(-8, 8, 384, device=cuda)
    a, b = h3p.split(x, blk=False), h3p.split(x, blk=True)
    assert b.blk and not a.blk
    for p in (0, 1):
        assert torch.equal(a.plane(p), b.plane(p))
    assert torch.equal(a.exps, b.exps)
    assert not torch.equal(a.planes, b.planes)  # (the storage order does differ)
    assert torch.equal(b.rows_slice(64, 160).unsplit(), a.unsplit()[64:160])


@pytest.mark.parametrize("ta,tb,M,N,K,ks", [(0, 1, 512, 384, 768, 1), (0, 0, 256, 768, 1024, 2),
                                            (1, 0, 384, 256, 2048, 4)])
def test_gemm_h3p_layouts_bitwise(cuda, ta, tb, M, N, K, ks):
    """Row-major and blocked operands, in all four layout pairs, give bitwise the same product (same
    values staged, same order of every sum)."""
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(6 + M + K)
    a = torch.randn((K, M) if ta else (M, K), device=cuda, generator=g)
    b = torch.randn((N, K) if tb else (K, N), device=cuda, generator=g)
    ref = h3p.gemm(h3p.split(a), h3p.split(b), ta, tb, ksplit=ks)
    for ab in (False, True):
        for bb in (False, True):
            out = h3p.gemm(h3p.split(a, blk=ab), h3p.split(b, blk=bb), ta, tb, ksplit=ks)
            assert torch.equal(out, ref), (ab, bb, (out - ref).abs().max().item())


def _operands(ta, tb, M, N, K, data, dev, g):
    if data == "uniform":
        a = torch.rand((K, M) if ta else (M, K), device=dev, generator=g) * 2 - 1
        b = torch.rand((N, K) if tb else (K, N), device=dev, generator=g) * 2 - 1
    else:
        # K >= 512: 6 decades of row scale inside every 32-row exponent block (beyond its 2^18 window:
        # the dot products' own fp32 rounding covers the bits the smallest rows lose); K = 64 (a head-
        # sized product, little accumulation to hide behind): 2 decades, inside the window
        dec = 6.0 if K >= 512 else 2.0
        a = _wide((K, M) if ta else (M, K), dev, g, dec) * 1e-5
        b = _wide((N, K) if tb else (K, N), dev, g, dec) * 1e3
    return a, b


@pytest.mark.parametrize("data", ["uniform", "wide"])
@pytest.mark.parametrize("ta,tb,M,N,K,ks", [(0, 1, 4096, 2304, 768, 1), (0, 0, 2048, 768, 3072, 2),
                                            (1, 0, 768, 3072, 4096, 4), (0, 1, 256, 384, 64, 1),
                                            (1, 0, 768, 768, 1024, 1), (0, 0, 512, 256, 2048, 1)])
def test_gemm_h3p_error_matches_fp32(cuda, data, ta, tb, M, N, K, ks):
    """All three Linear layouts, with and without split-K: error within 2x of exact-fp32 GEMMs
    against fp64 in units of |A|@|B|, including data with 6 decades of row scale (the per-block
    exponents keep every row's bits; the per-tensor h3 engine loses them beyond 2^18)."""
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(7 + M + N + K)
    a, b = _operands(ta, tb, M, N, K, data, cuda, g)
    At, Bt = (a.t() if ta else a), (b.t() if tb else b)
    ref = At.double() @ Bt.double()
    mag = At.double().abs() @ Bt.double().abs()
    out = torch.empty(M, N, device=cuda)

    def err(o):
        return float(((o.double() - ref).abs() / mag).max())

    torch.mm(At, Bt, out=out)
    e_blas = err(out)
    assert G._hip_gemm(a, b, ta, tb, out, fp32="native")
    e_nat = err(out)
    o = h3p.gemm(h3p.split(a), h3p.split(b), ta, tb, ksplit=ks)
    e = err(o)
    assert e <= 2.0 * max(e_blas, e_nat), (e, e_blas, e_nat)


@pytest.mark.parametrize("ta,tb", [(0, 1), (0, 0), (1, 0)])
def test_gemm_h3p_block_windows_beat_tensor_window(cuda, ta, tb):
    """32-row blocks of one operand scaled over 12 decades (2^40 across the tensor, small inside each
    block -- e.g. the masked-row structure of top-layer gradients): with a window per 32 x 32 block the
    error stays at fp32 level (within 2x of exact fp32 against fp64, per output row); a single
    per-tensor window (the h3 engine) loses the small blocks' bits."""
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(31)
    M, N, K = 1024, 768, 1024
    a = torch.randn((K, M) if ta else (M, K), device=cuda, generator=g)
    scales = torch.pow(10.0, -12.0 * torch.rand(a.shape[0] // 32, device=cuda, generator=g))
    a *= scales.repeat_interleave(32)[:, None]
    b = torch.randn((N, K) if tb else (K, N), device=cuda, generator=g) * 0.05
    At, Bt = (a.t() if ta else a), (b.t() if tb else b)
    ref = At.double() @ Bt.double()
    mag = At.double().abs() @ Bt.double().abs()
    out = torch.empty(M, N, device=cuda)

    def err(o):
        return float(((o.double() - ref).abs() / mag).max())

    assert G._hip_gemm(a, b, ta, tb, out, fp32="native")
    e_nat = err(out)
    e_new = err(h3p.gemm(h3p.split(a), h3p.split(b), ta, tb))
    assert G._hip_gemm(a, b, ta, tb, out, fp32="h3")
    e_old = err(out)
    print("block-scaled data: exact fp32 %.3g, h3p %.3g, per-tensor h3 %.3g" % (e_nat, e_new, e_old))
    assert e_new <= 2.0 * e_nat, (e_new, e_nat)


def test_gemm_h3p_nonfinite_propagates(cuda):
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(3)
    a = torch.randn(256, 256, device=cuda, generator=g)
    b = torch.randn(256, 256, device=cuda, generator=g)
    a[5, 17] = float("nan")
    o = h3p.gemm(h3p.split(a), h3p.split(b), 0, 1)
    assert torch.isnan(o[5]).all() and torch.isfinite(o[6]).all()
    a[5, 17] = float("inf")
    o = h3p.gemm(h3p.split(a), h3p.split(b), 0, 1)
    assert (~torch.isfinite(o[5])).all()


def test_gemm_h3p_epilogues(cuda):
    """bias, beta accumulation, split-K with bias + beta, the consumer-summed slabs, GELU (pre-
    activation out, planes out) and dGELU (planes out, bias-gradient column sums), against fp64."""
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(11)
    M, N, K = 512, 384, 768
    x = torch.randn(M, K, device=cuda, generator=g)
    w = torch.randn(N, K, device=cuda, generator=g) * 0.05
    bias = torch.randn(N, device=cuda, generator=g)
    hx, hw = h3p.split(x), h3p.split(w)
    ref = x.double() @ w.double().t()
    mag = x.double().abs() @ w.double().abs().t()

    def rel(o, r):
        return float(((o.double() - r).abs() / (mag + r.abs())).max())

    o = h3p.gemm(hx, hw, 0, 1, bias=bias, epi=h3p.EPI_BIAS)
    assert rel(o, ref + bias.double()) < 1e-6
    old = torch.randn(M, N, device=cuda, generator=g)
    o2 = old.clone()
    h3p.gemm(hx, hw, 0, 1, out=o2, beta=1.0)
    assert rel(o2, ref + old.double()) < 1e-6
    o3 = old.clone()
    h3p.gemm(hx, hw, 0, 1, out=o3, bias=bias, epi=h3p.EPI_BIAS, beta=1.0, ksplit=3)
    assert rel(o3, ref + old.double() + bias.double()) < 1e-6
    sl = h3p.gemm(hx, hw, 0, 1, ksplit=2, slab_only=True)
    assert sl.shape == (2, M, N) and rel(sl[0] + sl[1], ref) < 1e-6
    # GELU: pre-activation (un-biased) in aux, gelu(pre + bias) in fp32 and as planes
    pre = torch.empty(M, N, device=cuda)
    y = torch.empty(M, N, device=cuda)
    yp = h3p.empty(M, N, cuda)
    h3p.gemm(hx, hw, 0, 1, out=y, bias=bias, epi=h3p.EPI_GELU, aux=pre, planes_out=yp)
    assert rel(pre, ref) < 1e-6
    yref = _gelu_ref(pre.double() + bias.double())
    assert float((y.double() - yref).abs().max()) < 1e-6 * (1 + float(yref.abs().max()))
    assert torch.equal(yp.unsplit(), h3p.split(y).unsplit())
    # dGELU: dpre = (dy @ w) * gelu'(pre + bias); planes out only; db = column sums
    dy = torch.randn(M, N, device=cuda, generator=g)
    w2 = torch.randn(N, N, device=cuda, generator=g) * 0.05
    db = torch.zeros(N, device=cuda)
    part = torch.empty(M // 128, N, device=cuda)
    dp = h3p.empty(M, N, cuda)
    dpf = torch.empty(M, N, device=cuda)
    h3p.gemm(h3p.split(dy), h3p.split(w2), 0, 0, out=dpf, bias=bias, epi=h3p.EPI_DGELU, aux=pre, part=part,
             colsum=db, planes_out=dp)
    dref = (dy.double() @ w2.double()) * _gelu_grad_ref(pre.double() + bias.double())
    # (units of |dy| @ |w2|: gelu' itself crosses zero near -0.75, where its fp32 evaluation's absolute
    # error is all that is left of a relative one)
    dmag = dy.double().abs() @ w2.double().abs()
    assert float(((dpf.double() - dref).abs() / dmag).max()) < 1e-6
    assert torch.equal(dp.unsplit(), h3p.split(dpf).unsplit())
    assert float((db.double() - dref.sum(0)).abs().max()) < 1e-4 * float(dmag.sum(0).max())


def test_split_table_many_tensors(cuda):
    """One launch splitting several matrices (the weights): bit-identical to per-tensor splits."""
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(5)
    flat = torch.randn(768 * 2304 + 768 * 768 + 3072 * 768, device=cuda, generator=g)
    mats = [flat[:768 * 2304].view(2304, 768), flat[768 * 2304:768 * 3072].view(768, 768),
            flat[768 * 3072:].view(3072, 768)]
    dst = [h3p.empty(m.shape[0], m.shape[1], cuda) for m in mats]
    tab = h3p.SplitTable(list(zip(mats, dst)), cuda)
    tab.run()
    for m, d in zip(mats, dst):
        ref = h3p.split(m)
        assert torch.equal(d.planes, ref.planes) and torch.equal(d.exps, ref.exps)


def test_rows_slice_view(cuda):
    """A row window of an HP operand (the half-batch chains) computes the same rows as the whole."""
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(9)
    x = torch.randn(512, 768, device=cuda, generator=g)
    w = torch.randn(256, 768, device=cuda, generator=g)
    hx, hw = h3p.split(x), h3p.split(w)
    full = h3p.gemm(hx, hw, 0, 1)
    half = h3p.gemm(hx.rows_slice(256, 512), hw, 0, 1)
    assert torch.equal(full[256:], half)


@pytest.mark.parametrize("H,p,ns", [(768, 0.0, 2), (768, 0.1, 2), (1024, 0.1, 2), (768, 0.1, 4), (768, 0.1, 1),
                                     (768, 0.0, 3)])
def test_layernorm_h3p_planes(cuda, H, p, ns):
    """The LN forward / backward that write h3p planes: y, z, statistics and dz bitwise those of the
    plain kernels, the planes bitwise split(y) / split(da) (block exponents over 32-row blocks), the
    parameter-gradient partials (32-row blocks) equal to the plain kernel's to fp32 rounding.  ns: split-K
    slabs summed by the forward (1 / 2 / 4: the compile-time slab-count kernels, 3: the runtime loop);
    the 4-rows-per-workgroup forward runs with both slab paths (set_ln_fwd_ns)."""
    from hetseq_amd.ops import bert_ops as O
    from hetseq_amd.ops import h3p
    from hetseq_amd.ops._C import hip

    g = torch.Generator(device=cuda)
    g.manual_seed(H)
    rows = 256
    slabs = torch.randn(ns, rows, H, device=cuda, generator=g)
    bias = torch.randn(H, device=cuda, generator=g)
    resid = torch.randn(rows, H, device=cuda, generator=g)
    gamma = torch.rand(H, device=cuda, generator=g) + 0.5
    beta = torch.randn(H, device=cuda, generator=g)
    seed, off = 1234, 77
    ref = O.ln_fwd(slabs, gamma, beta, 1e-12, bias=bias, resid=resid, p=p, mode=1, seed=seed, off=off, row0=64)
    sp = h3p.split(ref[0])
    # every forward kernel (panel exchange at 8 / 4 rows per workgroup, one 32-row block of 16 / 8
    # waves), each called three times: the panel records must come back ready for the next call
    for mode, fns in ((0, 1), (1, 0), (16, 1), (8, 1), (1, 1)):
        hip().set_ln_h3p_waves(mode)
        hip().set_ln_fwd_ns(fns)
        try:
            for _ in range(3):
                outs = tuple(torch.full_like(t, float("nan")) for t in ref)
                hp = h3p.empty(rows, H, cuda)
                O.ln_fwd_h3p(slabs, gamma, beta, 1e-12, bias, resid, p, seed, off, outs, 64, hp)
                for a, b in zip(ref, outs):
                    assert torch.equal(a, b)
                assert torch.equal(hp.planes, sp.planes) and torch.equal(hp.exps, sp.exps), mode
        finally:
            hip().set_ln_h3p_waves(1)
            hip().set_ln_fwd_ns(1)
    # no bias / no residual (the MLM head's LayerNorm): the stand-in loads are selected away
    ref0 = O.ln_fwd(slabs, gamma, beta, 1e-12, p=p, mode=1, seed=seed, off=off, row0=64)
    for fns in (1, 0):
        hip().set_ln_fwd_ns(fns)
        try:
            outs = tuple(torch.full_like(t, float("nan")) for t in ref0)
            hp = h3p.empty(rows, H, cuda)
            O.ln_fwd_h3p(slabs, gamma, beta, 1e-12, None, None, p, seed, off, outs, 64, hp)
            for a, b in zip(ref0, outs):
                assert torch.equal(a, b), fns
        finally:
            hip().set_ln_fwd_ns(1)
    # backward
    dy = torch.randn(rows, H, device=cuda, generator=g)
    y, z, mean, rstd = ref
    dz, da, dg, db, dbias = O.ln_bwd(dy, z, mean, rstd, gamma, p, 1, seed, off, True, True)
    sp2 = h3p.split(da)
    for bmode in (1, 2, 0, 1):  # panel exchange at 8 / 4 rows per workgroup, the 32-row-block kernel
        hip().set_ln_bwd_coop(bmode)
        try:
            for _ in range(3):
                hp2 = h3p.empty(rows, H, cuda)
                dz2, dg2, db2, dbias2 = O.ln_bwd_h3p(dy, z, mean, rstd, gamma, p, seed, off, hp2)
                assert torch.equal(dz, dz2)
                assert torch.equal(hp2.planes, sp2.planes) and torch.equal(hp2.exps, sp2.exps), bmode
                for a, b in ((dg, dg2), (db, db2), (dbias, dbias2)):
                    assert float((a - b).abs().max()) <= 1e-5 * (1 + float(a.abs().max()))
        finally:
            hip().set_ln_bwd_coop(1)
    # no exchange timed out, and every record is back at rest (count 0; the other parity cleared)
    torch.cuda.synchronize()
    words = hip().panel_sync_words()
    for region in (0, 1):
        rec = O.panel_sync(cuda, rows + 64, region).view(-1, words)
        assert int(rec[:, 32].abs().sum()) == 0, "panel exchange timed out"
        assert int(rec[:, 16].abs().sum()) == 0


def test_panel_exchange_with_extreme_blocks(cuda):
    """Per-block exponents through the panel exchange when the 8-row workgroups of a panel disagree
    by many decades: rows 8-31 of every panel are constant (their LN output is beta, ~1e-6), rows
    0-7 are not (~1), and two column groups scale by 1e-20 / 1e20.  The exponent must be the
    panel's, so the planes are bitwise split(y)."""
    from hetseq_amd.ops import bert_ops as O
    from hetseq_amd.ops import h3p

    rows, H = 128, 768
    g = torch.Generator(device=cuda)
    g.manual_seed(3)
    a = torch.randn(rows, H, device=cuda, generator=g) * 1e-3
    a.view(-1, 32, H)[:, 8:] = 0.5
    gamma = torch.ones(H, device=cuda)
    beta = torch.randn(H, device=cuda, generator=g) * 1e-6
    gamma[:32] = 1e-20  # column blocks with tiny values
    gamma[32:64] = 1e20
    ref = O.ln_fwd(a, gamma, beta, 1e-12, mode=1)
    outs = tuple(torch.empty_like(t) for t in ref)
    hp = h3p.empty(rows, H, cuda)
    O.ln_fwd_h3p(a, gamma, beta, 1e-12, None, None, 0.0, 0, 0, outs, 0, hp)
    sp = h3p.split(ref[0])
    assert torch.equal(hp.planes, sp.planes) and torch.equal(hp.exps, sp.exps)


@pytest.mark.parametrize("S,p", [(128, 0.0), (128, 0.1), (512, 0.1)])
def test_attention_h3p_planes(cuda, S, p):
    """The h3 attention kernels that also write their outputs as h3p planes: ctx / dqkv bitwise those
    of the plain launch, the planes bitwise split(ctx) / split(dqkv)."""
    from hetseq_amd.ops import bert_ops as O
    from hetseq_amd.ops import h3p
    from hetseq_amd.ops._C import hip

    if hip().attn_fp32_mode() != 2:
        pytest.skip("fp32 attention engine is not h3")
    g = torch.Generator(device=cuda)
    g.manual_seed(S)
    B, NH, H = 4, 12, 768
    qkv = torch.randn(B * S, 3 * H, device=cuda, generator=g)
    bias = torch.randn(3 * H, device=cuda, generator=g) * 0.1
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[1, S - 40:] = 0
    ctx, (lse, dmask) = O.attn_fwd(qkv, mask, B, S, NH, p, 5, 9, bias=bias)
    outs = (torch.empty_like(ctx), torch.empty_like(lse), torch.empty_like(dmask) if dmask is not None else None)
    hp = h3p.empty(B * S, H, cuda)
    O.attn_fwd_h3p(qkv, mask, B, S, NH, p, 5, 9, bias, outs, 0, hp)
    assert torch.equal(outs[0], ctx) and torch.equal(outs[1], lse)
    sp = h3p.split(ctx)
    assert torch.equal(hp.planes, sp.planes) and torch.equal(hp.exps, sp.exps)
    dctx = torch.randn(B * S, H, device=cuda, generator=g)
    dq = O.attn_bwd(qkv, mask, ctx, dctx, (lse, dmask), B, S, NH, p, bias=bias)
    hq = h3p.empty(B * S, 3 * H, cuda)
    dq2 = O.attn_bwd_h3p(qkv, mask, ctx, dctx, (lse, dmask), B, S, NH, p, bias, hq)
    assert torch.equal(dq, dq2)
    sq = h3p.split(dq)
    assert torch.equal(hq.planes, sq.planes) and torch.equal(hq.exps, sq.exps)
    # planes only; the bias gradient's column partials from the planes
    hq3 = h3p.empty(B * S, 3 * H, cuda)
    assert O.attn_bwd_h3p(qkv, mask, ctx, dctx, (lse, dmask), B, S, NH, p, bias, hq3, fp32=False) is None
    assert torch.equal(hq3.planes, hq.planes) and torch.equal(hq3.exps, hq.exps)
    part = O.h3p_colpart(hq3, torch.full((B * S // 32, 3 * H), float("nan"), device=cuda))
    ref = dq.double().view(B * S // 32, 32, 3 * H).sum(1)
    err = (part.double() - ref).abs().max().item()
    assert err <= 1e-5 * (1.0 + ref.abs().max().item()), err


@pytest.mark.parametrize("rows,cols", [(64, 96), (256, 2304)])
def test_h3p_colpart_matches_planes(cuda, rows, cols):
    """h3p_colpart: per-32-row-panel column sums of what a blocked operand's planes hold ((hi + lo) 2^-e,
    exact in fp32), including column counts that leave a partial 256-column block."""
    from hetseq_amd.ops import bert_ops as O
    from hetseq_amd.ops import h3p

    g = torch.Generator(device=cuda)
    g.manual_seed(rows + cols)
    x = torch.randn(rows, cols, device=cuda, generator=g) * torch.logspace(-3, 3, cols, device=cuda)
    hp = h3p.split(x)
    part = O.h3p_colpart(hp, torch.full((rows // 32, cols), float("nan"), device=cuda))
    ref = x.double().view(rows // 32, 32, cols).sum(1)
    err = ((part.double() - ref).abs() / (1.0 + x.double().abs().view(rows // 32, 32, cols).sum(1))).max().item()
    assert err <= 1e-6, err
