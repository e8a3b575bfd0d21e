"""Meters: lazy device-tensor updates must match eager float updates (reference meters.py:4-65)."""
import torch

from hetseq_amd.meters import AverageMeter, StopwatchMeter, TimeMeter


def test_average_meter_lazy_matches_eager():
    lazy, eager = AverageMeter(), AverageMeter()
    for i in range(300):  # > 2 compactions of the pending list
        v, n = 0.5 * i, (i % 3) + 1
        lazy.update(torch.tensor(v, dtype=torch.float64), n)
        eager.update(v, n)
    assert len(lazy._pending) < 64
    assert abs(lazy.avg - eager.avg) < 1e-9
    assert lazy.count == eager.count and lazy.sum == eager.sum and lazy.val == eager.val


def test_average_meter_tensor_count():
    m = AverageMeter()
    m.update(torch.tensor(2.0), torch.tensor(4.0))
    m.update(1.0, 4)
    assert m.avg == 1.5 and m.count == 8


def test_time_meter_lazy_count():
    t = TimeMeter()
    for _ in range(10):
        t.update(torch.tensor(3.0, dtype=torch.float64))
    t.update(5)
    assert t.n == 35.0
    t.n = 7
    assert t.n == 7 and t.avg > 0


def test_stopwatch():
    s = StopwatchMeter()
    s.start()
    s.stop()
    assert s.n == 1 and s.sum >= 0
