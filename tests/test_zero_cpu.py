"""Sharded optimizer update (parallel/zero.py) on CPU/gloo, 2 processes.

A tiny BERT (unfused CPU path) trained 4 updates with gradient clipping through the flat-store DP
engine, once with the sharded update (each rank: Adam on its pieces of every bucket, all-gather) and
once with the whole update on every rank: the parameters agree to the rounding of the gradient norm
(summed over the shards in another order); the sharded run's consolidated optimizer state equals the
unsharded one's and loads into an unsharded optimizer (checkpoint round trip).
"""
import socket

import pytest
import torch
import torch.distributed as dist
import multiprocessing as mp

pytestmark = pytest.mark.slow


def _model():
    from hetseq_amd.models.bert import BertConfig, BertForPreTraining

    torch.manual_seed(0)
    cfg = BertConfig(vocab_size_or_config_json_file=96, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                     intermediate_size=128)
    return BertForPreTraining(cfg), cfg


def _batch(rank, step, cfg):
    g = torch.Generator().manual_seed(100 * rank + step)
    B, S = 4, 16
    ids = torch.randint(0, cfg.vocab_size, (B, S), generator=g)
    tt = torch.zeros(B, S, dtype=torch.long)
    mask = torch.ones(B, S, dtype=torch.long)
    labels = torch.full((B, S), -1, dtype=torch.long)
    labels[:, 3] = torch.randint(0, cfg.vocab_size, (B,), generator=g)
    labels[:, 7] = torch.randint(0, cfg.vocab_size, (B,), generator=g)
    nsp = torch.randint(0, 2, (B,), generator=g)
    return ids, tt, mask, labels, nsp


def _worker(rank, port, shard, q, world=2):
    try:
        _work(rank, port, shard, q, world)
    except BaseException:
        import traceback

        q.put(("error", rank, traceback.format_exc()))
        raise


def _work(rank, port, shard, q, world=2):
    from argparse import Namespace

    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime.flat import FlatParamStore

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, world_size=world, rank=rank)
    torch.set_num_threads(2)
    model, cfg = _model()
    model.train(False)
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    ddp = FlatDDP(model, store, bucket_cap_mb=1, shard_optimizer=shard)
    # "auto" on c10d (gloo): the replicated update (sharding pays only on the native engine)
    assert (store.shard is not None) == (shard is True)
    if shard is True:
        # one bucket per update chunk; every element of the buffer owned by exactly one rank's piece
        # or by both ranks' (replicated) tails
        assert len(ddp.buckets) == len([c for c in store.chunks])
    opt = _Adam(Namespace(lr=[5e-3], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                list(model.parameters()), store)
    norms = []
    for step in range(4):
        opt.zero_grad()
        loss = ddp(*_batch(rank, step, cfg))
        loss.backward()
        opt.multiply_grads(0.5)
        norms.append(float(opt.clip_grad_norm(0.05)))  # (small: the clip is active)
        opt.step()
    opt.consolidate()
    sd = opt.state_dict()
    # (numpy through the queue: torch tensors would travel as shared memory the exiting worker frees)
    q.put((shard, rank, store.param.numpy().copy(), norms,
           {k: sd["state"][0][k].numpy().copy() for k in ("exp_avg", "exp_avg_sq")},
           torch.cat([sd["state"][i]["exp_avg_sq"].reshape(-1) for i in sorted(sd["state"])]).numpy().copy()))
    dist.destroy_process_group()


def _run(shard, world=2):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, shard, q, world)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for o in out:
        assert o[0] != "error", o[2]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    conv = lambda x: torch.from_numpy(x) if hasattr(x, "dtype") else x  # noqa: E731
    return {r[1]: (r[0], r[1], conv(r[2]), r[3], {k: conv(v) for k, v in r[4].items()}, conv(r[5])) for r in out}


@pytest.mark.parametrize("world", [2, pytest.param(8, marks=pytest.mark.skipif(
    __import__("os").environ.get("HETSEQ_TEST_W8") != "1", reason="8 gloo ranks: HETSEQ_TEST_W8=1"))])
def test_sharded_update_matches_unsharded_and_round_trips(world):
    from argparse import Namespace

    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.runtime.flat import FlatParamStore

    full = _run("auto", world)  # (auto on gloo = the replicated update)
    sh = _run(True, world)
    # every rank holds the same parameters after the all-gather
    assert all(torch.equal(sh[0][2], sh[r][2]) for r in range(1, world))
    for r in range(world):
        p_full, p_sh = full[r][2], sh[r][2]
        assert torch.allclose(p_sh, p_full, rtol=1e-5, atol=1e-6), (p_sh - p_full).abs().max()
        for a, b in zip(full[r][3], sh[r][3]):
            assert abs(a - b) <= 1e-5 * abs(a), (a, b)
        # the consolidated moments are the unsharded ones
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.allclose(sh[r][4][k], full[r][4][k], rtol=1e-4, atol=1e-9)
        assert torch.allclose(sh[r][5], full[r][5], rtol=1e-4, atol=1e-12)
    # checkpoint round trip: the sharded run's state loads into an unsharded optimizer
    model, _ = _model()
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    opt = _Adam(Namespace(lr=[5e-3], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                list(model.parameters()), store)
    n = len(opt.param_list)
    state = {"state": {}, "param_groups": opt.state_dict()["param_groups"]}
    off = 0
    flat = sh[0][5]
    for i, p in enumerate(opt.param_list):
        state["state"][i] = {"step": 4, "exp_avg": torch.zeros_like(p), "exp_avg_sq": flat[off:off + p.numel()].view(p.shape)}
        off += p.numel()
    opt.load_state_dict(state)
    assert opt.step_count == 4 and len(opt.param_list) == n
    got = torch.cat([v["exp_avg_sq"].reshape(-1) for _, v in sorted(opt.state_dict()["state"].items())])
    assert torch.equal(got, flat)
