"""The native layer program (ops/layer_prog.py, csrc/kernels/layer_prog.cpp) against the Python layer
it replaces: the same kernels with the same arguments on the same streams, so training is BITWISE
equal -- losses, parameters and Adam moments -- with dropout on, the two half-batch forward chains or
one chain, two micro-batches per update (the accumulating weight-gradient path) and the staged
update re-splitting the weight planes between steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(cuda, use_prog, B, S, update_freq, steps=3):
    from argparse import Namespace

    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.runtime import rng
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    G.set_fp32_mode("h3p")
    bert_ops.LAYER_PROG = use_prog
    try:
        model, cfg = _tiny(cuda)
        model.train()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        opt = _Adam(Namespace(lr=[1e-3], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                    list(model.parameters()), store)
        opt.staged = True
        b = _batch(cuda, B, S, cfg.vocab_size)
        assert model.bert._can_fuse(b[0])
        losses = []
        for step in range(steps):
            opt.zero_grad(lazy=True)
            for micro in range(update_freq):
                rng.set_seed(100 + 10 * step + micro)
                loss = model(*b)
                loss.backward()
                losses.append(loss.detach().clone())
            opt.multiply_grads(0.5)
            opt.clip_grad_norm(1.0)
            opt.step()
        opt.state_dict()  # (waits for the staged update)
        torch.cuda.synchronize()
        if use_prog:
            assert any(p.rows == B * S for blk in model.bert.encoder.layer
                       for p in blk.__dict__.get("_hs_progs", {}).values())
        return (torch.stack(losses), store.param.clone(), opt._state["exp_avg"].clone(),
                opt._state["exp_avg_sq"].clone())
    finally:
        bert_ops.LAYER_PROG = True


@pytest.mark.parametrize("B,S,update_freq", [(16, 64, 1), (16, 64, 2), (4, 64, 1)])
def test_layer_program_matches_python_layer(cuda, B, S, update_freq):
    ref = _train(cuda, False, B, S, update_freq)
    got = _train(cuda, True, B, S, update_freq)
    for x, y in zip(ref, got):
        assert torch.equal(x, y), (x - y).abs().max().item()
