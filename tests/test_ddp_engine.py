"""FlatDDP engine unit tests (CPU, gloo, 2 processes).

Regression for the readiness signal: a fused Function that accumulates its
weight gradient directly into the flat buffer and returns None must still be
counted exactly once (post-accumulate-grad hooks fire for None grads), so no
bucket is all-reduced before all of its gradients are written.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import multiprocessing as mp

pytestmark = pytest.mark.slow


class _DirectLinear(torch.autograd.Function):
    """y = x @ W^T whose backward writes dW into the flat store and returns None."""

    @staticmethod
    def forward(ctx, x, w, store):
        ctx.save_for_backward(x, w)
        ctx.store = store
        return x @ w.t()

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        ctx.store.grad_view(w).add_(dy.t() @ x)
        return dy @ w, None, None


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 16)
        self.w = torch.nn.Parameter(torch.randn(16, 16) * 0.1)
        self.b = torch.nn.Linear(16, 4)
        self.store = None

    def forward(self, x):
        h = torch.tanh(self.a(x))
        h = _DirectLinear.apply(h, self.w, self.store)
        return self.b(h).pow(2).sum()


def _worker(rank, port, q):
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime.flat import FlatParamStore

    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, world_size=2, rank=rank)
    torch.manual_seed(0)
    net = _Net()
    store = FlatParamStore(net)
    net.store = store
    ddp = FlatDDP(net, store, bucket_cap_mb=0.0001)  # one parameter per bucket
    x = torch.randn(5, 8, generator=torch.Generator().manual_seed(rank))
    for micro in range(2):  # update_freq 2: first micro-batch under no_sync
        ctx = ddp.no_sync() if micro == 0 else torch.enable_grad()
        with ctx:
            ddp(x * (micro + 1)).backward()
    q.put((rank, store.grad.numpy().copy(), len(ddp.buckets)))
    dist.destroy_process_group()


def test_direct_grads_reduce_exactly_once():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (torch.from_numpy(g), nb)) for r, g, nb in [q.get(timeout=120) for _ in range(2)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    g0, nb = res[0]
    g1, _ = res[1]
    assert nb == 3  # tiny cap: several buckets, launched in order during backward
    assert torch.equal(g0, g1)
    # reference: sum over ranks of the locally accumulated gradients (single process)
    from hetseq_amd.runtime.flat import FlatParamStore

    total = torch.zeros_like(g0)
    for rank in range(2):
        torch.manual_seed(0)
        net = _Net()
        st = FlatParamStore(net)
        net.store = st
        x = torch.randn(5, 8, generator=torch.Generator().manual_seed(rank))
        net(x).backward()
        net(2 * x).backward()
        total += st.grad
    assert torch.allclose(g0, total, atol=1e-5, rtol=1e-5)
