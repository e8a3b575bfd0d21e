"""Synchronisation logic of the half-batch forward chains (runtime/streams.py ``fwd_chain`` /
``fwd_halves`` / ``chain_keep``), on the CPU with the HIP calls recorded instead of issued: inside a
chain the second stream is forked once and joined once, at the chain's end; outside a chain every
block forks and joins; tensors kept for the second stream live until the join."""
import types

import pytest
import torch

from hetseq_amd.runtime import streams


class _Rec(object):
    def __init__(self):
        self.calls = []

    def stream_wait(self, waiter, signal):
        self.calls.append((waiter, signal))


@pytest.fixture
def fake(monkeypatch):
    import hetseq_amd.ops._C as C

    rec = _Rec()
    side = types.SimpleNamespace(cuda_stream=222, device_index=0, stream_id=0, device_type=1)
    monkeypatch.setattr(C, "hip", lambda: rec)
    monkeypatch.setattr(C, "stream_handle", lambda: 111)
    monkeypatch.setattr(streams, "fwd2", lambda device: side)
    # the second half switches the current stream: keep it a no-op here
    monkeypatch.setattr(torch._C, "_cuda_getCurrentStream", lambda idx: (0, 0, 1), raising=False)
    monkeypatch.setattr(torch._C, "_cuda_setStream", lambda **kw: None, raising=False)
    monkeypatch.setattr(streams, "FWD_CHAIN", True)
    streams._chain.update(depth=0, forked=None)
    streams._chain["keep"].clear()
    yield rec
    streams._chain.update(depth=0, forked=None)
    streams._chain["keep"].clear()


def _layer(dev, keep=None):
    with streams.fwd_halves(dev) as halves:
        for _ in halves:
            pass
    if keep is not None:
        streams.chain_keep(keep)


def test_every_block_forks_and_joins_outside_a_chain(fake):
    for _ in range(3):
        _layer("cpu")
    assert fake.calls == [(222, 111), (111, 222)] * 3


def test_chain_orders_each_layer_one_way_and_joins_at_its_end(fake):
    """Inside a chain every layer orders the second stream after the current one (its half may
    write into blocks the current stream's allocator re-issued) -- one-way waits only: the current
    stream meets the second chain once, at the end."""
    t = torch.zeros(4)
    with streams.fwd_chain("cpu"):
        for _ in range(12):
            _layer("cpu", keep=t)
        assert fake.calls == [(222, 111)] * 12  # second stream waits; the current stream never does
        assert len(streams._chain["keep"]) == 12  # the layers' tensors stay referenced
    assert fake.calls == [(222, 111)] * 12 + [(111, 222)]
    assert streams._chain["forked"] is None and not streams._chain["keep"]


def test_chain_forks_once_without_the_per_layer_wait(fake, monkeypatch):
    monkeypatch.setattr(streams, "FWD_CHAIN_FORK", False)
    with streams.fwd_chain("cpu"):
        for _ in range(12):
            _layer("cpu")
        assert fake.calls == [(222, 111)]
    assert fake.calls == [(222, 111), (111, 222)]


def test_chain_join_before_an_unsplit_layer(fake):
    with streams.fwd_chain("cpu"):
        _layer("cpu")
        streams.chain_join("cpu")  # an unsplit layer reads both halves: the chains meet first
        assert fake.calls == [(222, 111), (111, 222)]
        _layer("cpu")  # the next split layer forks again
    assert fake.calls == [(222, 111), (111, 222), (222, 111), (111, 222)]


def test_chain_off_behaves_like_no_chain(fake, monkeypatch):
    monkeypatch.setattr(streams, "FWD_CHAIN", False)
    with streams.fwd_chain("cpu"):
        _layer("cpu")
        _layer("cpu")
    assert fake.calls == [(222, 111), (111, 222)] * 2


def test_exception_inside_a_chain_joins(fake):
    with pytest.raises(RuntimeError):
        with streams.fwd_chain("cpu"):
            with streams.fwd_halves("cpu") as halves:
                for _ in halves:
                    raise RuntimeError("boom")
    assert fake.calls[-1] == (111, 222)
    assert streams._chain["forked"] is None
