"""Training-log bars (reference: progress_bar.py:13-138).

Formats:
* ``simple`` -- the reference's text lines, byte for byte:
  ``| epoch 001:      5 / 100 loss=1.234, ...`` every ``--log-interval``
  items (after the consumer handled item i, never for i = 0), and
  ``| epoch 001 | loss 1.234 | ...`` for end-of-epoch summaries;
* ``none`` -- silent;
* ``json`` -- one JSON object per logged step (the reference names it but
  never defines it, Q22).
``--json-log FILE`` additionally appends every ``log()`` call as a JSON line
(numbers only), for benchmark harnesses.  Stats handed to ``log()`` may hold
lazy device meters: the text is only rendered when a line is actually printed,
so logging never forces a host-device sync.
"""
import json
from collections import OrderedDict
from numbers import Number

from hetseq_amd.meters import AverageMeter, StopwatchMeter, TimeMeter

_TEXT = (
    (AverageMeter, lambda m: "{:.3f}".format(m.avg)),
    (TimeMeter, lambda m: "{:g}".format(round(m.avg))),
    (StopwatchMeter, lambda m: "{:.4f}".format(m.sum)),
)


def format_stat(stat):
    """Text of one stat: numbers with ``%g``, meters by their reference rule, anything else unchanged."""
    if isinstance(stat, Number):
        return "{:g}".format(stat)
    for cls, fmt in _TEXT:
        if isinstance(stat, cls):
            return fmt(stat)
    return stat


def _value(stat):
    """Plain JSON-able value of one stat (meters -> their average / total)."""
    if isinstance(stat, (AverageMeter, TimeMeter)):
        return stat.avg
    if isinstance(stat, StopwatchMeter):
        return stat.sum
    if not isinstance(stat, Number) and hasattr(stat, "__float__"):
        return float(stat)
    return stat


def _rendered(stats):
    return OrderedDict((k, str(format_stat(v)).strip()) for k, v in stats.items())


class progress_bar(object):
    """Base bar: wraps an iterable, numbers its items from the iterable's ``offset`` and calls
    ``_after(i, size)`` once the consumer is done with item ``i``."""

    json_sink = None

    def __init__(self, iterable, epoch=None, prefix=None):
        self.iterable = iterable
        self.offset = getattr(iterable, "offset", 0)
        self.epoch = epoch
        parts = []
        if epoch is not None:
            parts.append("| epoch {:03d}".format(epoch))
        if prefix is not None:
            parts.append(" | {}".format(prefix))
        self.prefix = "".join(parts)

    def __len__(self):
        return len(self.iterable)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __iter__(self):
        size = len(self.iterable)
        for i, item in enumerate(self.iterable, start=self.offset):
            yield item
            self._after(i, size)

    def _after(self, i, size):
        pass

    def _due(self, i):
        return getattr(self, "stats", None) is not None and i > 0 and self.log_interval is not None \
            and i % self.log_interval == 0

    def log(self, stats, tag="", step=None):
        """Record intermediate stats (printed at the next log-interval boundary)."""
        self._sink(stats, step)

    def print(self, stats, tag="", step=None):
        """Print end-of-epoch stats."""

    def _sink(self, stats, step):
        if not self.json_sink:
            return
        rec = OrderedDict(epoch=self.epoch, step=step)
        rec.update((k, v) for k, v in ((k, _value(v)) for k, v in stats.items())
                   if v is None or isinstance(v, Number))
        with open(self.json_sink, "a") as f:
            f.write(json.dumps(rec) + "\n")


class noop_progress_bar(progress_bar):
    """Iterates without printing (``--log-format none`` / ``--no-progress-bar``)."""


class _Deferred(object):
    """Stats whose text is rendered on first use (keeps lazy device meters lazy)."""

    def __init__(self, stats):
        self._stats, self._text = stats, None

    def text(self):
        if self._text is None:
            self._text = _rendered(self._stats)
        return self._text


class simple_progress_bar(progress_bar):
    """Plain text lines for non-TTY logs."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix)
        self.log_interval = log_interval
        self.stats = None

    def _after(self, i, size):
        if self._due(i):
            body = ", ".join("{}={}".format(k, v) for k, v in self.stats.text().items())
            print("{}:  {:5d} / {:d} {}".format(self.prefix, i, size, body), flush=True)

    def log(self, stats, tag="", step=None):
        self.stats = _Deferred(stats)
        self._sink(stats, step)

    def print(self, stats, tag="", step=None):
        body = " | ".join("{} {}".format(k, v) for k, v in _rendered(stats).items())
        print("{} | {}".format(self.prefix, body), flush=True)


class json_progress_bar(progress_bar):
    """One JSON object per logged step on stdout."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix)
        self.log_interval = log_interval
        self.stats = None

    def _after(self, i, size):
        if self._due(i):
            rec = OrderedDict(epoch=self.epoch, update=i)
            for k, v in self.stats.items():
                v = _value(v)
                rec[k] = round(v, 6) if isinstance(v, float) else v
            print(json.dumps(rec), flush=True)

    def log(self, stats, tag="", step=None):
        self.stats = stats
        self._sink(stats, step)

    def print(self, stats, tag="", step=None):
        rec = OrderedDict(epoch=self.epoch)
        rec.update((k, _value(v)) for k, v in stats.items())
        print(json.dumps(rec), flush=True)


_BARS = {"none": noop_progress_bar, "simple": simple_progress_bar, "json": json_progress_bar}


def build_progress_bar(args, iterator, epoch=None, prefix=None, default="simple", no_progress_bar="none"):
    if args.log_format is None:
        args.log_format = no_progress_bar if args.no_progress_bar else default
    cls = _BARS.get(args.log_format)
    if cls is None:
        raise ValueError("Unknown log format: {}".format(args.log_format))
    bar = cls(iterator, epoch, prefix) if cls is noop_progress_bar else cls(iterator, epoch, prefix, args.log_interval)
    if getattr(args, "json_log", None):
        bar.json_sink = args.json_log
    return bar
