"""Meters (reference: meters.py:4-65).

Same classes and semantics.  ``AverageMeter`` additionally accepts 0-d
device tensors lazily: values are only converted to Python floats when read
(``avg``/``sum``), so the training loop never forces a host sync just to
update a meter.
"""
import time

import torch


def _f(v):
    if torch.is_tensor(v):
        return float(v.detach().cpu().item())
    return v


class _Folded(object):
    """A compacted run of lazy updates: sum of val*n and sum of n (device tensors or numbers)."""

    __slots__ = ("total", "count")

    def __init__(self, total, count):
        self.total, self.count = total, count


class AverageMeter(object):
    """Computes and stores the average and current value"""

    def __init__(self):
        self.reset()

    def reset(self):
        self._val = 0
        self._sum = 0
        self.count = 0
        self._pending = []

    def update(self, val, n=1):
        if torch.is_tensor(val) or torch.is_tensor(n):
            self._pending.append((val, n))
            if len(self._pending) >= 64:
                self._compact()
        else:
            self._fold(val, n)
        self._last = (val, n)

    def _compact(self):
        """Fold the pending device values into one (sum, count) pair on the device (no host sync)."""
        last = self._pending[-1]
        tot, cnt = 0, 0
        for v, n in self._pending[:-1]:
            if isinstance(v, _Folded):
                tot, cnt = tot + v.total, cnt + v.count
            else:
                tot, cnt = tot + v * n, cnt + n
        self._pending = [(_Folded(tot, cnt), 1), last]

    def _fold(self, val, n):
        self._val = val
        self._sum += val * n
        self.count += n

    def _flush(self):
        if self._pending:
            pend, self._pending = self._pending, []
            for v, n in pend:
                if isinstance(v, _Folded):
                    self._sum += _f(v.total)
                    self.count += _f(v.count)
                else:
                    self._fold(_f(v), _f(n))

    @property
    def val(self):
        self._flush()
        return self._val

    @property
    def sum(self):
        self._flush()
        return self._sum

    @property
    def avg(self):
        self._flush()
        return self._sum / self.count if self.count else 0

    def state_dict(self):
        self._flush()
        return {"val": self._val, "sum": self._sum, "count": self.count}

    def load_state_dict(self, sd):
        self.reset()
        self._val, self._sum, self.count = sd["val"], sd["sum"], sd["count"]

    def __getstate__(self):
        self._flush()
        d = dict(self.__dict__)
        d.pop("_last", None)
        return d


class TimeMeter(object):
    """Computes the average occurrence of some event per second"""

    def __init__(self, init=0):
        self.reset(init)

    def reset(self, init=0):
        self.init = init
        self.start = time.time()
        self._n = 0
        self._dn = None  # lazily accumulated device count (no per-update host sync)

    def update(self, val=1):
        if torch.is_tensor(val):
            self._dn = val.detach().clone() if self._dn is None else self._dn.add_(val)
        else:
            self._n += val

    @property
    def n(self):
        if self._dn is not None:
            self._n += _f(self._dn)
            self._dn = None
        return self._n

    @n.setter
    def n(self, v):
        self._n, self._dn = v, None

    @property
    def avg(self):
        return self.n / self.elapsed_time

    @property
    def elapsed_time(self):
        return self.init + (time.time() - self.start)


class StopwatchMeter(object):
    """Computes the sum/avg duration of some event in seconds"""

    def __init__(self):
        self.reset()

    def start(self):
        self.start_time = time.time()

    def stop(self, n=1):
        if self.start_time is not None:
            delta = time.time() - self.start_time
            self.sum += delta
            self.n += n
            self.start_time = None

    def reset(self):
        self.sum = 0
        self.n = 0
        self.start_time = None

    @property
    def avg(self):
        return self.sum / self.n if self.n else 0
