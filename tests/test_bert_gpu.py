"""Whole-model checks on the GPU: fused HIP path vs the torch-op reference path."""
import copy
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _tiny(cuda, H=256, L=2, NH=4, V=1000):
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining

    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=V, hidden_size=H, num_hidden_layers=L, num_attention_heads=NH,
                     intermediate_size=4 * H)
    return BertForPreTraining(cfg).to(cuda), cfg


def _batch(cuda, B, S, V, P=10):
    g = torch.Generator(device="cpu").manual_seed(1)
    ids = torch.randint(0, V, (B, S), generator=g).to(cuda)
    tt = (torch.arange(S) > S // 2).long().expand(B, S).contiguous().to(cuda)
    mask = torch.ones(B, S, dtype=torch.long)
    mask[0, S - 9:] = 0
    labels = torch.full((B, S), -1, dtype=torch.long)
    for b in range(B):
        pos = torch.randperm(S - 2, generator=g)[:P] + 1
        labels[b, pos] = torch.randint(0, V, (P,), generator=g)
    nsp = torch.randint(0, 2, (B,), generator=g)
    return ids, tt, mask.to(cuda), labels.to(cuda), nsp.to(cuda)


def test_fused_matches_reference_loss_and_grads(cuda):
    model, cfg = _tiny(cuda)
    model.eval()  # dropout off -> deterministic comparison
    ref = copy.deepcopy(model)
    ref._hs_disable_fused = True
    ref.bert._hs_disable_fused = True
    model.max_predictions_per_seq = 10
    batch = _batch(cuda, 4, 64, cfg.vocab_size)
    assert model.bert._can_fuse(batch[0])
    l1 = model(*batch)
    os.environ["HETSEQ_DISABLE_FUSED"] = "1"
    try:
        l2 = ref(*batch)
    finally:
        del os.environ["HETSEQ_DISABLE_FUSED"]
    assert abs(l1.item() - l2.item()) < 1e-4 * abs(l2.item()) + 1e-5, (l1.item(), l2.item())
    l1.backward()
    l2.backward()
    worst = 0.0
    for (n, p1), (_, p2) in zip(model.named_parameters(), ref.named_parameters()):
        d = (p1.grad - p2.grad).abs().max().item()
        scale = p2.grad.abs().max().item() + 1e-6
        worst = max(worst, d / scale)
        assert d <= 2e-3 * scale + 1e-6, (n, d, scale)


@pytest.mark.parametrize("side", [False, True])
def test_direct_flat_grads_match_autograd_grads(cuda, side):
    """With a flat store attached, fused kernels accumulate grads in place; values must match.
    Run the way a real update does: zero_grad() opens the fresh-gradient window, so with the side
    stream on the first backward STORES the weight / fused QKV-bias / tied-decoder gradients (the
    embedding rows then add onto the decoder's store) and the second backward accumulates."""
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore

    old = streams.enabled()
    streams.set_enabled(side)
    try:
        model, cfg = _tiny(cuda)
        model.eval()
        model.max_predictions_per_seq = 10
        ref = copy.deepcopy(model)
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        batch = _batch(cuda, 4, 64, cfg.vocab_size)
        store.grad.fill_(123.0)  # stale values: only a store or zero_grad may remove them
        store.zero_grad()
        for _ in range(2):  # two micro-batches: the first stores (side), the second accumulates
            model(*batch).backward()
            ref(*batch).backward()
        torch.cuda.synchronize()
        for (n, p1), (_, p2) in zip(model.named_parameters(), ref.named_parameters()):
            assert p1.grad.data_ptr() == store.grad_view(p1).data_ptr(), n
            d = (p1.grad - p2.grad).abs().max().item()
            assert d <= 1e-4 * (p2.grad.abs().max().item() + 1e-6) + 1e-7, (n, d)
    finally:
        streams.set_enabled(old)


@pytest.mark.parametrize("side,micro", [(True, 1), (True, 2), (False, 1)])
def test_lazy_zero_grad_matches_full_zero(cuda, side, micro):
    """A lazy zero_grad (runtime/flat.py: only the regions the backward does not overwrite are cleared)
    gives bitwise the gradients of a full zero_grad, from a buffer full of stale values: with the side
    stream the first backward stores the covered regions, a second micro-batch accumulates onto them;
    without it every covered writer accumulates after ensure_zero."""
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore

    old = streams.enabled()
    streams.set_enabled(side)
    try:
        model, cfg = _tiny(cuda)
        model.eval()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        batch = _batch(cuda, 4, 64, cfg.vocab_size)
        store.zero_grad()
        model(*batch).backward()  # registers the covered regions (fused layers, tied decoder)
        assert store._cover, "no store-covered gradient regions registered"
        grads = {}
        for lazy in (False, True):
            store.grad.fill_(123.0)
            store.zero_grad(lazy=lazy)
            for _ in range(micro):
                model(*batch).backward()
            store.flush_lazy()
            torch.cuda.synchronize()
            grads[lazy] = store.grad.clone()
        assert torch.equal(grads[True], grads[False])
    finally:
        streams.set_enabled(old)


@pytest.mark.parametrize("kind", ["odd_seq", "unlabelled"])
def test_lazy_zero_grad_then_unfused_backward(cuda, kind):
    """A fused step registers the store-covered regions; a later lazy zero_grad followed by a batch
    the fused path does not serve (S not a multiple of 32, or no labels: autograd accumulates into the
    covered weight / tied-decoder gradients) must give the gradients of a full zero_grad -- the
    non-fused forward clears the pending regions first (bert.py _flush_lazy_grads)."""
    from hetseq_amd.runtime.flat import FlatParamStore

    model, cfg = _tiny(cuda)
    model.eval()
    model.max_predictions_per_seq = 10
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    store.zero_grad()
    model(*_batch(cuda, 4, 64, cfg.vocab_size)).backward()  # fused: registers the covered regions
    assert store._cover
    if kind == "odd_seq":
        batch = _batch(cuda, 4, 40, cfg.vocab_size)
        run = lambda: model(*batch).backward()  # noqa: E731
    else:
        ids, tt, mask = _batch(cuda, 4, 64, cfg.vocab_size)[:3]
        run = lambda: sum(t.float().square().sum() for t in model(ids, tt, mask)).backward()  # noqa: E731
    grads = {}
    for lazy in (False, True):
        store.grad.fill_(123.0)
        store.zero_grad(lazy=lazy)
        run()
        store.flush_lazy()
        torch.cuda.synchronize()
        grads[lazy] = store.grad.clone()
    assert torch.equal(grads[True], grads[False])


def test_lazy_zero_grad_flushes_unclaimed_regions(cuda):
    """Covered regions no writer claimed read as zero once the gradients are read (flush_lazy), and
    ensure_zero clears a pending region exactly once."""
    from hetseq_amd.runtime.flat import FlatParamStore

    model, _ = _tiny(cuda)
    store = FlatParamStore(model)
    ps = [p for p in model.parameters() if p.dim() == 2 and p.numel() % 4 == 0][:3]
    store.cover(*(store.grad_view(p) for p in ps))
    store.grad.fill_(5.0)
    store.zero_grad(lazy=True)
    torch.cuda.synchronize()
    covered = sum(p.numel() for p in ps)
    assert int((store.grad != 0).sum()) == covered  # only the covered regions kept their stale values
    store.ensure_zero(store.grad_view(ps[0]))
    assert float(store.grad_view(ps[0]).abs().max()) == 0.0
    store.grad_view(ps[0]).fill_(1.0)  # "accumulated" after ensure_zero: not cleared again
    store.ensure_zero(store.grad_view(ps[0]))
    assert float(store.grad_view(ps[0]).min()) == 1.0
    store.mark_stored(store.grad_view(ps[1]))
    store.flush_lazy()  # clears ps[2] only
    assert float(store.grad_view(ps[2]).abs().max()) == 0.0
    assert float(store.grad_view(ps[1]).min()) == 5.0


def test_fused_train_step_with_store_and_dropout(cuda):
    from argparse import Namespace

    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.runtime import rng
    from hetseq_amd.runtime.flat import FlatParamStore

    model, cfg = _tiny(cuda)
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    model.max_predictions_per_seq = 10
    opt = _Adam(Namespace(lr=[1e-3], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                list(model.parameters()), store)
    batch = _batch(cuda, 8, 128, cfg.vocab_size)
    losses = []
    for step in range(8):
        rng.set_seed(100 + step)
        opt.zero_grad()
        loss = model(*batch)
        loss.backward()
        # flat grads are the param .grad storage
        p0 = next(model.parameters())
        assert p0.grad.data_ptr() >= store.grad.data_ptr()
        opt.multiply_grads(1.0)
        opt.clip_grad_norm(5.0)
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0], losses


def test_bf16_mode_runs_and_tracks_fp32(cuda):
    from hetseq_amd.runtime.flat import FlatParamStore

    model, cfg = _tiny(cuda)
    model.eval()
    model.max_predictions_per_seq = 10
    m32 = copy.deepcopy(model)
    store = FlatParamStore(model, shadow_dtype=torch.bfloat16)
    model.attach_store(store, torch.bfloat16)
    batch = _batch(cuda, 4, 128, cfg.vocab_size)
    l16 = model(*batch)
    l32 = m32(*batch)
    assert torch.isfinite(l16)
    assert abs(l16.item() - l32.item()) < 0.05 * abs(l32.item()), (l16.item(), l32.item())
    l16.backward()
    assert torch.isfinite(store.grad).all()


def test_bf16_padded_decoder_matches_library(cuda):
    """bf16: the tied decoder's three products on the plane kernels over the padded vocabulary
    (BertForPreTraining._head_bf16_pad) give the loss and gradients of the library products on the
    unpadded shapes, to bf16 rounding -- and the padded weight copy follows the updates."""
    import hetseq_amd.models.bert as MB
    from hetseq_amd.runtime.flat import FlatParamStore

    model, cfg = _tiny(cuda)
    model.eval()
    # cap = 4 x 32 = 128 rows in both runs (no row padding of its own): the MLM transform's products run
    # on the same kernels either way, so only the three decoder products differ between the runs
    model.max_predictions_per_seq = 32
    ref = copy.deepcopy(model)
    stores = []
    for m in (model, ref):
        st = FlatParamStore(m, shadow_dtype=torch.bfloat16)
        m.attach_store(st, torch.bfloat16)
        stores.append(st)
    batch = _batch(cuda, 4, 128, cfg.vocab_size)
    old = MB.HEAD_BF16_PAD
    try:
        MB.HEAD_BF16_PAD = True
        l1 = model(*batch)
        l1.backward()
        assert model.__dict__.get("_hs_head_bf16") is not None
        MB.HEAD_BF16_PAD = False
        l2 = ref(*batch)
        l2.backward()
    finally:
        MB.HEAD_BF16_PAD = old
    assert abs(l1.item() - l2.item()) <= 2e-3 * abs(l2.item()), (l1.item(), l2.item())
    g1, g2 = stores[0].grad.double(), stores[1].grad.double()
    assert torch.isfinite(g1).all()
    # per parameter, relative to its largest entry floored at 1 % of the model's largest gradient entry:
    # the two runs round differently in bf16 (fp32 accumulation order of the decoder products, then the
    # bf16 data gradient), and parameters whose gradient is that small hold mostly such noise
    gmax = g2.abs().max().item()
    worst, where = 0.0, None
    for (n, p1), (_, p2) in zip(model.named_parameters(), ref.named_parameters()):
        o1, o2 = stores[0].offset(p1), stores[1].offset(p2)
        a, b = g1[o1:o1 + p1.numel()], g2[o2:o2 + p2.numel()]
        r = (a - b).abs().max().item() / max(b.abs().max().item(), 1e-2 * gmax)
        worst, where = (r, n) if r > worst else (worst, where)
    assert worst <= 2e-2, (worst, where)
    wd = model.cls.predictions.decoder.weight
    off = stores[0].offset(wd)
    n = wd.numel()
    dg1, dg2 = g1[off:off + n], g2[off:off + n]
    assert (dg1 - dg2).abs().max().item() <= 2e-2 * dg2.abs().max().item()  # the decoder's own gradient


def test_base_model_param_count(cuda):
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining

    cfg = BertConfig(30522)
    m = BertForPreTraining(cfg)
    assert sum(p.numel() for p in m.parameters()) == 110106428
    assert len(m.state_dict()) == 207


def _grad_report(model, ref):
    """Worst per-parameter gradient difference relative to the oracle's largest entry of that
    parameter -- floored at 1e-3 of the model's largest gradient entry: the key biases' gradient
    is exactly zero in exact arithmetic (a per-query constant shift of the scores cancels in the
    softmax), so both paths hold rounding noise there and a ratio of noises means nothing."""
    gmax = max(p.grad.abs().max().item() for p in ref.parameters())
    worst, where = 0.0, None
    for (n, p1), (_, p2) in zip(model.named_parameters(), ref.named_parameters()):
        d = (p1.grad.double() - p2.grad.double()).abs().max().item()
        r = d / max(p2.grad.abs().max().item(), 1e-3 * gmax)
        if r > worst:
            worst, where = r, n
    return worst, where


def _row_grad_report(model, ref):
    """Worst per-ROW gradient difference of the 2-D parameters: each row's largest |difference|
    relative to the oracle's largest entry of that row (rows whose largest entry is below 1e-6 of the
    parameter's are rounding noise in both paths and skipped) -- small rows are judged on their own
    scale, not hidden under the parameter's largest entry."""
    worst, where = 0.0, None
    for (n, p1), (_, p2) in zip(model.named_parameters(), ref.named_parameters()):
        if p1.dim() != 2:
            continue
        g1, g2 = p1.grad.double(), p2.grad.double()
        rmax = g2.abs().amax(dim=1)
        keep = rmax > 1e-6 * rmax.max()
        if not keep.any():
            continue
        r = ((g1 - g2).abs().amax(dim=1)[keep] / rmax[keep]).max().item()
        if r > worst:
            worst, where = r, n
    return worst, where


@pytest.mark.parametrize("engine", ["x6", "h3", "h3p"])
def test_bert_base_shape_matches_reference_1e4(cuda, engine):
    """BERT-base (H 768, L 12, 12 heads, S 128, B 8), dropout off: the fused fp32 path -- in-kernel
    split engine (six split-bf16 products, x6; three split-fp16 products with per-tensor scales,
    h3; three fp16-plane products with 32x32 block exponents, h3p) -- against the fp32 torch-op oracle (the
    reference module graph, bert_modeling.py:819-888).  Loss to 1e-5 relative; every parameter's
    gradient within 1e-4 of the oracle's largest gradient entry of that parameter."""
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.runtime.flat import FlatParamStore

    G.set_fp32_mode(engine)  # (conftest restores the default after the test)
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=30522)
    model = BertForPreTraining(cfg).to(cuda)
    model.eval()
    model.max_predictions_per_seq = 20
    ref = copy.deepcopy(model)
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    batch = _batch(cuda, 8, 128, cfg.vocab_size, P=20)
    assert model.bert._can_fuse(batch[0])
    l1 = model(*batch)
    os.environ["HETSEQ_DISABLE_FUSED"] = "1"
    try:
        l2 = ref(*batch)
        l2.backward()
    finally:
        del os.environ["HETSEQ_DISABLE_FUSED"]
    l1.backward()
    assert abs(l1.item() - l2.item()) <= 1e-5 * abs(l2.item()), (l1.item(), l2.item())
    worst, where = _grad_report(model, ref)
    rworst, rwhere = _row_grad_report(model, ref)
    print("bert-base fused vs oracle (engine=%s): loss %.8g vs %.8g, worst grad rel %.3g at %s, "
          "worst per-row rel %.3g at %s" % (engine, l1.item(), l2.item(), worst, where, rworst, rwhere))
    assert worst <= 1e-4, (worst, where)
    if engine == "h3p":
        assert rworst <= 1e-3, (rworst, rwhere)


@pytest.mark.parametrize("engine", ["x6", "h3", "h3p"])
def test_trajectory_200_updates_tracks_reference(cuda, monkeypatch, engine):
    """200 Adam updates of a tiny BERT, fused (flat store, fused Adam) vs the torch-op oracle with
    the reference Adam math (optim.py:162-231), identical seeds and batches, dropout off: the two
    loss curves stay within 1e-4 relative of each other at every update (both fp32 GEMM engines)."""
    from argparse import Namespace

    from hetseq_amd.ops import gemm as G
    from hetseq_amd.optim.optimizers import AdamReference, _Adam
    from hetseq_amd.runtime.flat import FlatParamStore

    G.set_fp32_mode(engine)

    model, cfg = _tiny(cuda, H=256, L=2, NH=4, V=1000)
    model.eval()
    model.max_predictions_per_seq = 10
    ref = copy.deepcopy(model)
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    opt = _Adam(Namespace(lr=[1e-4], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                list(model.parameters()), store)
    ropt = AdamReference(ref.parameters(), lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    batches = [_batch(cuda, 4, 64, cfg.vocab_size) for _ in range(4)]
    for i in range(4):  # distinct batches
        torch.manual_seed(100 + i)
        ids = torch.randint(0, cfg.vocab_size, batches[i][0].shape, device=cuda)
        batches[i] = (ids,) + batches[i][1:]
    worst = 0.0
    for step in range(200):
        b = batches[step % 4]
        opt.zero_grad()
        l1 = model(*b)
        l1.backward()
        opt.step()
        ropt.zero_grad()
        os.environ["HETSEQ_DISABLE_FUSED"] = "1"
        try:
            l2 = ref(*b)
            l2.backward()
        finally:
            del os.environ["HETSEQ_DISABLE_FUSED"]
        ropt.step()
        rel = abs(l1.item() - l2.item()) / abs(l2.item())
        worst = max(worst, rel)
        assert rel <= 1e-4, (step, l1.item(), l2.item())
    print("200-update trajectory (%s): worst loss rel diff %.3g" % (engine, worst))


@pytest.mark.parametrize("engine", ["h3", "h3p"])
def test_bert_base_trajectory_50_updates(cuda, engine):
    """BERT-base (H 768, L 12, S 128, B 8) for 50 Adam updates, fused (flat store, fused Adam, the
    given fp32 product engine) vs the fp32 torch-op oracle with the reference Adam math, identical
    batches, dropout off: the loss curves stay within 1e-4 relative at every update."""
    from argparse import Namespace

    from hetseq_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.optim.optimizers import AdamReference, _Adam
    from hetseq_amd.runtime.flat import FlatParamStore

    G.set_fp32_mode(engine)
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=30522)
    model = BertForPreTraining(cfg).to(cuda)
    model.eval()
    model.max_predictions_per_seq = 20
    ref = copy.deepcopy(model)
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    opt = _Adam(Namespace(lr=[1e-4], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                list(model.parameters()), store)
    ropt = AdamReference(ref.parameters(), lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)
    batches = []
    for i in range(4):
        b = _batch(cuda, 8, 128, cfg.vocab_size, P=20)
        torch.manual_seed(200 + i)
        batches.append((torch.randint(0, cfg.vocab_size, b[0].shape, device=cuda),) + b[1:])
    worst = 0.0
    for step in range(50):
        b = batches[step % 4]
        opt.zero_grad()
        l1 = model(*b)
        l1.backward()
        opt.step()
        ropt.zero_grad()
        os.environ["HETSEQ_DISABLE_FUSED"] = "1"
        try:
            l2 = ref(*b)
            l2.backward()
        finally:
            del os.environ["HETSEQ_DISABLE_FUSED"]
        ropt.step()
        rel = abs(l1.item() - l2.item()) / abs(l2.item())
        worst = max(worst, rel)
        assert rel <= 1e-4, (step, l1.item(), l2.item())
    print("BERT-base 50-update trajectory (%s): worst loss rel diff %.3g" % (engine, worst))


@pytest.mark.parametrize("engine", ["h3p", "h3"])
def test_staged_update_matches_unstaged(cuda, engine):
    """The staged update (optimizer chunks on their own stream overlapped with the next forward,
    per-layer h3p weight planes re-split by update hooks, zero_grad queued behind the update) trains
    bitwise like the unstaged one: same losses, parameters and moments after 6 steps, dropout on,
    half-batch forward chains, gradient scale and clipping as the controller applies them."""
    from argparse import Namespace

    from hetseq_amd.ops import gemm as G
    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.runtime import rng
    from hetseq_amd.runtime.flat import FlatParamStore

    G.set_fp32_mode(engine)
    runs = []
    for staged in (False, False, True):  # (the first pair: the unstaged step is deterministic)
        model, cfg = _tiny(cuda)
        model.train()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        assert store.chunks is not None and len(store.chunks) == cfg.num_hidden_layers + 2
        opt = _Adam(Namespace(lr=[1e-3], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                    list(model.parameters()), store)
        opt.staged = staged
        b = _batch(cuda, 16, 64, cfg.vocab_size)
        assert model.bert._can_fuse(b[0])
        losses = []
        for step in range(6):
            rng.set_seed(100 + step)  # (the fused kernels' dropout seeds, as the controller sets them)
            opt.zero_grad(lazy=True)
            loss = model(*b)
            loss.backward()
            opt.multiply_grads(0.5)
            opt.clip_grad_norm(1.0)
            opt.step()
            assert store.staged_pending() == staged
            losses.append(loss.detach().clone())
        sd = opt.state_dict()  # (waits for the staged update)
        assert not store.staged_pending()
        torch.cuda.synchronize()
        runs.append((torch.stack(losses), store.param.clone(), opt._state["exp_avg"].clone(),
                     opt._state["exp_avg_sq"].clone(), sd["state"][0]["exp_avg"].clone()))
    print("losses unstaged", runs[0][0].tolist(), "\nlosses unstaged", runs[1][0].tolist(),
          "\nlosses staged  ", runs[2][0].tolist())
    for other in (runs[1], runs[2]):
        for x, y in zip(runs[0], other):
            assert torch.equal(x, y), (x - y).abs().max().item()


def test_lamb_hip_step_matches_cpu_math(cuda):
    """The fused LAMB kernel (per-tensor trust ratios over the flat store) against the
    _step_cpu math on identical copies: parameters and both moments over several steps."""
    from argparse import Namespace

    from hetseq_amd.optim.optimizers import _Lamb
    from hetseq_amd.runtime.flat import FlatParamStore

    args = Namespace(lr=[2e-3], adam_betas="(0.9,0.999)", adam_eps=1e-6, weight_decay=0.01)
    torch.manual_seed(5)
    net = torch.nn.Sequential(torch.nn.Linear(64, 96), torch.nn.LayerNorm(96), torch.nn.Linear(96, 10)).to(cuda)
    net2 = copy.deepcopy(net)
    s1, s2 = FlatParamStore(net), FlatParamStore(net2)
    o1, o2 = _Lamb(args, list(net.parameters()), s1), _Lamb(args, list(net2.parameters()), s2)
    covered = torch.zeros(s1.numel, dtype=torch.bool, device=cuda)  # parameter elements (not alignment gaps)
    for q in net.parameters():
        covered[s1.offset(q):s1.offset(q) + q.numel()] = True
    for step in range(5):
        g = torch.randn_like(s1.grad) * (0.1 + step) * covered
        s1.grad.copy_(g)
        s2.grad.copy_(g)
        o1.step_count += 1
        o2.step_count += 1
        gm = torch.full((1,), 0.5, device=cuda)
        o1._step_hip(gm)
        o2._step_cpu(gm)
        torch.cuda.synchronize()
        for a, b, what in ((s1.param, s2.param, "param"), (o1._state["exp_avg"], o2._state["exp_avg"], "m"),
                           (o1._state["exp_avg_sq"], o2._state["exp_avg_sq"], "v")):
            torch.testing.assert_close(a[covered], b[covered], rtol=2e-6, atol=1e-7,
                                       msg=lambda m: "%s step %d: %s" % (what, step, m))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layer_forward_half_batch_streams_match(cuda, monkeypatch, dtype):
    """The encoder layer forward as two half-batch chains on two streams writes the same tensors as
    the one-chain forward: LN and attention dropout masks drawn by whole-batch index (the backward
    regenerates the LN ones that way; the attention keep bits are bitwise the same), every saved
    tensor equal to GEMM tolerance (bf16: to bf16 rounding -- the halves' GEMM sites may pick other K
    splits than the whole batch's)."""
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.runtime.flat import FlatParamStore

    torch.manual_seed(5)
    cfg = BertConfig(vocab_size_or_config_json_file=512, hidden_size=768, num_hidden_layers=1,
                     num_attention_heads=12, intermediate_size=3072)
    model = BertForPreTraining(cfg).cuda()
    bf = dtype == torch.bfloat16
    model.attach_store(FlatParamStore(model, shadow_dtype=torch.bfloat16) if bf else FlatParamStore(model), dtype)
    W = model.bert.encoder.layer[0]._weights()
    B, S = 16, 128
    x = torch.randn(B * S, 768, device=cuda).to(dtype)
    mask = torch.ones(B, S, dtype=torch.int64, device=cuda)
    mask[3, 100:] = 0
    c = (B, S, 12, 0.1, 0.1, 1e-12, ((7, 0), (7, 256), (7, 512)))  # hidden and attention dropout on
    monkeypatch.setattr(bert_ops, "_FWD_SPLIT", True)
    assert bert_ops._fwd_split_ok(x, mask, W, c)
    h_s, sv_s = bert_ops._layer_forward(x, mask, W, c, save=True)
    monkeypatch.setattr(bert_ops, "_FWD_SPLIT", False)
    h_1, sv_1 = bert_ops._layer_forward(x, mask, W, c, save=True)
    torch.cuda.synchronize()
    names = ["qkv", "ctx", "lse", "dmask", "z1", "m1", "r1", "h1", "f1pre", "f1", "z2", "m2", "r2", "x", "ctx2"]
    for n, a, b in zip(names, sv_s, sv_1):
        if a is None:
            assert b is None
            continue
        assert a.dtype == b.dtype, n
        a, b = a.float() if a.is_floating_point() else a, b.float() if b.is_floating_point() else b
        tol = (2e-2 if bf else 1e-5) * float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= tol, n
    h_s, h_1 = h_s.float(), h_1.float()
    assert float((h_s - h_1).abs().max()) <= (2e-2 if bf else 1e-5) * float(h_1.abs().max())  # (another mask: O(1))
    assert torch.equal(sv_s[3], sv_1[3])  # attention keep bits


def test_forward_chain_with_scratch_frees_matches_unchained(cuda, monkeypatch):
    """Half-batch forward chains across layers, with large compute-stream scratch buffers freed
    between layers (their blocks go back to the pool the next layer's whole-batch outputs come from):
    the chained no-grad forward is bitwise the unchained one (streams.FWD_CHAIN_FORK orders the
    second chain after each layer's allocations)."""
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining, BertLayer
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore

    if not streams.enabled():
        pytest.skip("side stream disabled")
    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=1024, hidden_size=768, num_hidden_layers=4,
                     num_attention_heads=12, intermediate_size=3072)
    model = BertForPreTraining(cfg).to(cuda)
    model.eval()
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    ids = torch.randint(0, 1024, (16, 128), device=cuda)
    tt, mask = torch.zeros_like(ids), torch.ones_like(ids)
    orig = BertLayer.fused

    def noisy(self, *a, **k):
        junk = torch.empty(16 * 128 * 3072 * 2, device=cuda)
        junk.fill_(float("nan"))  # a compute-stream kernel on the block, then the block is freed
        del junk
        return orig(self, *a, **k)

    monkeypatch.setattr(BertLayer, "fused", noisy)
    outs = {}
    for chain in (False, True):
        monkeypatch.setattr(streams, "FWD_CHAIN", chain)
        with torch.no_grad():
            seq, _ = model.bert(ids, tt, mask, output_all_encoded_layers=False)
        torch.cuda.synchronize()
        outs[chain] = seq.clone()
    assert torch.isfinite(outs[True]).all()
    assert torch.equal(outs[True], outs[False])


def test_checkpoint_activations_with_split_forward_matches(cuda):
    """--checkpoint-activations on the fused path: the backward recomputes each layer's forward (as
    two half-batch chains, the second on the side stream that already holds the later layers'
    weight-gradient GEMMs) and must give the stored-activation run's loss and gradients."""
    from hetseq_amd.ops import bert_ops
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore

    old = streams.enabled()
    streams.set_enabled(True)
    try:
        model, cfg = _tiny(cuda, H=256, L=3)
        model.eval()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        batch = _batch(cuda, 16, 64, cfg.vocab_size)
        x = torch.zeros(16 * 64, 256, device=cuda)
        W = model.bert.encoder.layer[0]._weights()
        assert bert_ops._fwd_split_ok(x, batch[2], W, (16, 64, 4, 0.0, 0.0, 1e-12, ((0, 0),) * 3))
        outs = []
        for ck in (False, True):
            store.grad.zero_()
            loss = model(*batch, checkpoint_activations=ck)
            loss.backward()
            torch.cuda.synchronize()
            outs.append((loss.item(), store.grad.clone()))
        (l0, g0), (l1, g1) = outs
        assert abs(l0 - l1) <= 1e-6 * abs(l0)
        assert float((g0 - g1).abs().max()) <= 1e-6 * float(g0.abs().max())
    finally:
        streams.set_enabled(old)
