"""Step bookkeeping on CPU: the ordering points of runtime/streams.py with the HIP calls stubbed
(consecutive forks inside ``streams.coalesced()`` record one event -- the compute stream pays
~6.5 us of GPU time per ordering point, profiles/r3_forks.md -- and a fork after the block records
again), and the flat store's fresh-gradient window (runtime/flat.py claim_fresh)."""
import pytest

from hetseq_amd.runtime import streams


class _Hip(object):
    def __init__(self):
        self.waits = []

    def stream_wait(self, waiter, signal):
        self.waits.append((waiter, signal))


class _Side(object):
    cuda_stream = 22


@pytest.fixture
def stub(monkeypatch):
    import hetseq_amd.ops._C as C

    h = _Hip()
    monkeypatch.setattr(C, "hip", lambda: h)
    monkeypatch.setattr(C, "stream_handle", lambda: 11)
    monkeypatch.setattr(streams, "side", lambda device: _Side())
    monkeypatch.setitem(streams._state, "queued", True)  # as inside a backward (no engine callback)
    monkeypatch.setitem(streams._state, "coalesce", 0)
    yield h
    streams._KEEP.clear()


def test_each_fork_records_outside_a_block(stub):
    for _ in range(3):
        streams.fork(None)
    assert stub.waits == [(22, 11)] * 3


def test_coalesced_forks_share_the_first_event(stub):
    with streams.coalesced():
        for _ in range(3):
            streams.fork(None)
    assert stub.waits == [(22, 11)]
    streams.fork(None)  # compute work may have been enqueued since: a new ordering point
    assert len(stub.waits) == 2


def test_coalescing_switch_off_records_every_fork(stub, monkeypatch):
    monkeypatch.setattr(streams, "COALESCE", False)
    with streams.coalesced():
        streams.fork(None)
        streams.fork(None)
    assert len(stub.waits) == 2


def test_nested_blocks_restore_the_outer_state(stub):
    with streams.coalesced():
        streams.fork(None)
        with streams.coalesced():
            streams.fork(None)  # a new block: records
        streams.fork(None)
    assert len(stub.waits) == 2
    assert streams._state["coalesce"] == 0


def test_fresh_gradients_claimed_for_one_backward_only():
    """FlatParamStore.claim_fresh: True throughout the first backward after zero_grad (weight
    gradients may store instead of accumulate), False from the end of that backward on."""
    import torch

    from hetseq_amd.runtime.flat import FlatParamStore

    lin = torch.nn.Linear(4, 3)
    store = FlatParamStore(lin)
    seen = []

    class Probe(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            seen.append((store.claim_fresh(), store.claim_fresh()))
            return g

    x = torch.randn(2, 4, requires_grad=True)
    assert not store.claim_fresh()  # nothing zeroed yet: accumulate
    store.zero_grad()
    Probe.apply(x).sum().backward()
    assert seen[-1] == (True, True) and not store.grads_zero
    Probe.apply(x).sum().backward()  # a second micro-batch accumulates
    assert seen[-1] == (False, False)
