"""Progress bars / loggers (reference: progress_bar.py:13-138).

``simple`` reproduces the reference line format byte-for-byte:
``| epoch 001:      5 / 100 loss=..., ppl=...``.  ``none`` is silent.
``json`` (defined here; the reference names it but never implements it, Q22)
prints one JSON object per logged step.  An optional JSON-lines sink
(``--json-log``) records every logged step for benchmark harnesses.
"""
import json
import sys
from collections import OrderedDict
from numbers import Number

from hetseq_amd.meters import AverageMeter, StopwatchMeter, TimeMeter


def build_progress_bar(args, iterator, epoch=None, prefix=None, default="simple", no_progress_bar="none"):
    if args.log_format is None:
        args.log_format = no_progress_bar if args.no_progress_bar else default
    if args.log_format == "none":
        bar = noop_progress_bar(iterator, epoch, prefix)
    elif args.log_format == "simple":
        bar = simple_progress_bar(iterator, epoch, prefix, args.log_interval)
    elif args.log_format == "json":
        bar = json_progress_bar(iterator, epoch, prefix, args.log_interval)
    else:
        raise ValueError("Unknown log format: {}".format(args.log_format))
    sink = getattr(args, "json_log", None)
    if sink:
        bar.json_sink = sink
    return bar


def format_stat(stat):
    if isinstance(stat, Number):
        stat = "{:g}".format(stat)
    elif isinstance(stat, AverageMeter):
        stat = "{:.3f}".format(stat.avg)
    elif isinstance(stat, TimeMeter):
        stat = "{:g}".format(round(stat.avg))
    elif isinstance(stat, StopwatchMeter):
        stat = "{:.4f}".format(stat.sum)
    return stat


def _plain(stat):
    if isinstance(stat, AverageMeter):
        return stat.avg
    if isinstance(stat, TimeMeter):
        return stat.avg
    if isinstance(stat, StopwatchMeter):
        return stat.sum
    if not isinstance(stat, Number) and hasattr(stat, "__float__"):
        return float(stat)
    return stat


class progress_bar(object):
    """Abstract class for progress bars."""

    json_sink = None

    def __init__(self, iterable, epoch=None, prefix=None):
        self.iterable = iterable
        self.offset = getattr(iterable, "offset", 0)
        self.epoch = epoch
        self.prefix = ""
        if epoch is not None:
            self.prefix += "| epoch {:03d}".format(epoch)
        if prefix is not None:
            self.prefix += " | {}".format(prefix)

    def __len__(self):
        return len(self.iterable)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __iter__(self):
        raise NotImplementedError

    def log(self, stats, tag="", step=None):
        raise NotImplementedError

    def print(self, stats, tag="", step=None):
        raise NotImplementedError

    def _str_commas(self, stats):
        return ", ".join(key + "=" + stats[key].strip() for key in stats.keys())

    def _str_pipes(self, stats):
        return " | ".join(key + " " + stats[key].strip() for key in stats.keys())

    def _format_stats(self, stats):
        postfix = OrderedDict(stats)
        for key in postfix.keys():
            postfix[key] = str(format_stat(postfix[key]))
        return postfix

    def _sink(self, stats, step):
        if self.json_sink:
            rec = OrderedDict(epoch=self.epoch, step=step)
            for k, v in stats.items():
                v = _plain(v)
                if isinstance(v, Number) or v is None:
                    rec[k] = v
            with open(self.json_sink, "a") as f:
                f.write(json.dumps(rec) + "\n")


class noop_progress_bar(progress_bar):
    def __iter__(self):
        for obj in self.iterable:
            yield obj

    def log(self, stats, tag="", step=None):
        self._sink(stats, step)

    def print(self, stats, tag="", step=None):
        pass


class simple_progress_bar(progress_bar):
    """A minimal logger for non-TTY environments."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix)
        self.log_interval = log_interval
        self.stats = None

    def __iter__(self):
        size = len(self.iterable)
        for i, obj in enumerate(self.iterable, start=self.offset):
            yield obj
            if self.stats is not None and i > 0 and self.log_interval is not None and i % self.log_interval == 0:
                postfix = self._str_commas(self.stats)
                print("{}:  {:5d} / {:d} {}".format(self.prefix, i, size, postfix), flush=True)

    def log(self, stats, tag="", step=None):
        # formatting resolves lazy (device) meters; only do it when a line will be printed
        self._raw = stats
        self.stats = _LazyFormat(self, stats)
        self._sink(stats, step)

    def print(self, stats, tag="", step=None):
        postfix = self._str_pipes(self._format_stats(stats))
        print("{} | {}".format(self.prefix, postfix), flush=True)


class _LazyFormat(object):
    """Formats the stats only when the progress bar actually prints them."""

    def __init__(self, bar, stats):
        self._bar, self._stats, self._cache = bar, stats, None

    def _get(self):
        if self._cache is None:
            self._cache = self._bar._format_stats(self._stats)
        return self._cache

    def keys(self):
        return self._get().keys()

    def __getitem__(self, k):
        return self._get()[k]


class json_progress_bar(progress_bar):
    """One JSON object per logged step on stdout."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix)
        self.log_interval = log_interval
        self.stats = None
        self._step = None

    def __iter__(self):
        for i, obj in enumerate(self.iterable, start=self.offset):
            yield obj
            if self.stats is not None and i > 0 and self.log_interval is not None and i % self.log_interval == 0:
                rec = OrderedDict(epoch=self.epoch, update=i)
                for k, v in self.stats.items():
                    v = _plain(v)
                    rec[k] = round(v, 6) if isinstance(v, float) else v
                print(json.dumps(rec), flush=True)
                sys.stdout.flush()

    def log(self, stats, tag="", step=None):
        self.stats = stats
        self._sink(stats, step)

    def print(self, stats, tag="", step=None):
        rec = OrderedDict(epoch=self.epoch)
        for k, v in stats.items():
            rec[k] = _plain(v)
        print(json.dumps(rec), flush=True)
