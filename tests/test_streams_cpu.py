"""Ordering-point bookkeeping of runtime/streams.py, on CPU with the HIP calls stubbed: consecutive
forks inside ``streams.coalesced()`` record one event (the compute stream pays ~6.5 us of GPU time
per ordering point, profiles/r3_forks.md), and a fork after the block records again."""
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
