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
        else:
            self._fold(val, n)
        self._last = (val, n)

    def _fold(self, val, n):
        self._val = val
        self._sum += val * n
        self.count += n

    def _flush(self):
        if self._pending:
            pend, self._pending = self._pending, []
            for v, n in pend:
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
        self.n = 0

    def update(self, val=1):
        self.n += _f(val)

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
