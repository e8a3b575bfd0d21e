"""BMUF (``--use-bmuf``, parallel/ddp.py:BMUF) on CPU/gloo, 2 processes.

The reference only exposes the flag and lets ranks train independently
(controller.py:77,324).  Here every ``sync_interval`` updates the
ranks average their parameters and apply a block-momentum filtered step.
Checked: the constructor broadcast, the no-op between syncs, identical
parameters on every rank after a sync, and the update math
(global <- global - smoothed, smoothed = bm * smoothed + blr * (global - avg),
params <- global - bm * smoothed) against a single-process recomputation.
"""
import socket

import multiprocessing as mp
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.slow

BM, BLR = 0.5, 1.0


def _worker(rank, port, q):
    from hetseq_amd.parallel.ddp import BMUF
    from hetseq_amd.runtime.flat import FlatParamStore

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, world_size=2, rank=rank)
    torch.manual_seed(rank)  # different init per rank: the constructor must broadcast rank 0's
    net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Linear(5, 3))
    store = FlatParamStore(net)
    bmuf = BMUF(store, block_momentum=BM, block_lr=BLR, sync_interval=2)
    out = {"init": store.param.clone()}
    steps = []
    for k in range(4):  # a local "optimizer step" that differs per rank
        with torch.no_grad():
            store.param.add_(0.1 * (rank + 1) * (k + 1))
        pre = store.param.clone()
        bmuf.after_step()
        steps.append((pre, store.param.clone()))
    out["steps"] = steps
    q.put((rank, {"init": out["init"].numpy(), "steps": [(a.numpy(), b.numpy()) for a, b in steps]}))
    dist.destroy_process_group()


def test_bmuf_block_momentum_sync():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    t = lambda a: torch.from_numpy(a).double()  # noqa: E731
    assert torch.equal(t(res[0]["init"]), t(res[1]["init"]))  # broadcast from rank 0
    glob = t(res[0]["init"])
    smooth = torch.zeros_like(glob)
    for k in range(4):
        pre0, post0 = map(t, res[0]["steps"][k])
        pre1, post1 = map(t, res[1]["steps"][k])
        if k % 2 == 0:  # sync_interval 2: the first update of each block is local only
            assert torch.equal(pre0, post0) and torch.equal(pre1, post1)
            continue
        assert torch.allclose(post0, post1, atol=1e-6)
        avg = (pre0 + pre1) / 2
        smooth = BM * smooth + BLR * (glob - avg)
        glob = glob - smooth
        expect = glob - BM * smooth
        assert torch.allclose(post0, expect, atol=1e-5), (post0 - expect).abs().max()
