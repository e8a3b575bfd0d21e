"""Progress bars (reference progress_bar.py:13-138): the ``simple`` line formats, the
log-interval rule (print after the consumer handled item i, only for i > 0), the
resume offset, the ``json`` bar the reference names but never defines (Q22), and the
JSON-lines sink."""
import argparse
import json
from collections import OrderedDict

import torch

from hetseq_amd.meters import AverageMeter, StopwatchMeter, TimeMeter
from hetseq_amd.progress_bar import build_progress_bar, format_stat


def _args(fmt, interval=2, sink=None, no_bar=False):
    return argparse.Namespace(log_format=fmt, no_progress_bar=no_bar, log_interval=interval, json_log=sink)


class _Offset(list):
    offset = 4  # a CountingIterator resumed mid-epoch


def test_format_stat_matches_reference_rules():
    m = AverageMeter()
    m.update(1.23456, 1)
    sw = StopwatchMeter()
    sw.sum = 2.5
    assert format_stat(3) == "3" and format_stat(0.5) == "0.5" and format_stat(1e-7) == "1e-07"
    assert format_stat(m) == "1.235"
    assert format_stat(sw) == "2.5000"
    t = TimeMeter()
    assert format_stat(t) == "0"
    lazy = AverageMeter()
    lazy.update(torch.tensor(0.25, dtype=torch.float64), 1)  # device-style lazy meter
    assert format_stat(lazy) == "0.250"


def test_simple_bar_lines_and_interval(capsys):
    items = list(range(5))
    bar = build_progress_bar(_args("simple", interval=2), items, epoch=1)
    seen = []
    for i in bar:
        seen.append(i)
        st = OrderedDict(loss=AverageMeter(), num_updates=i + 1)
        st["loss"].update(0.5 * i, 1)
        bar.log(st, tag="train", step=i + 1)
    out = capsys.readouterr().out.splitlines()
    assert seen == items
    # printed after items 2 and 4 (never at i = 0), with the stats logged for that item
    assert out == ["| epoch 001:      2 / 5 loss=1.000, num_updates=3",
                   "| epoch 001:      4 / 5 loss=2.000, num_updates=5"]
    bar.print(OrderedDict(loss=1.5, wall=12), tag="train")
    assert capsys.readouterr().out == "| epoch 001 | loss 1.5 | wall 12\n"


def test_simple_bar_resume_offset(capsys):
    bar = build_progress_bar(_args("simple", interval=3), _Offset([10, 11]), epoch=2, prefix="train")
    for i in bar:
        bar.log({"loss": 1.0})
    # enumerate starts at the iterator's offset: the items are numbered 4 and 5, neither a multiple of 3
    assert capsys.readouterr().out == ""
    bar = build_progress_bar(_args("simple", interval=5), _Offset([10, 11]), epoch=2, prefix="train")
    for i in bar:
        bar.log({"loss": 1.0})
    assert capsys.readouterr().out == "| epoch 002 | train:      5 / 2 loss=1\n"


def test_none_and_no_progress_bar_are_silent(capsys):
    a = _args(None, no_bar=True)
    bar = build_progress_bar(a, [1, 2, 3], epoch=1)
    assert a.log_format == "none"
    for _ in bar:
        bar.log({"loss": 1.0})
    bar.print({"loss": 1.0})
    assert capsys.readouterr().out == ""


def test_json_bar_and_sink(tmp_path, capsys):
    sink = tmp_path / "log.jsonl"
    bar = build_progress_bar(_args("json", interval=1, sink=str(sink)), [0, 1, 2], epoch=3)
    for i in bar:
        m = AverageMeter()
        m.update(0.1 * (i + 1), 1)
        bar.log(OrderedDict(loss=m, lr=1e-4, name="x"), step=i + 1)
    lines = [json.loads(l) for l in capsys.readouterr().out.splitlines()]
    assert [l["update"] for l in lines] == [1, 2]
    assert lines[0]["epoch"] == 3 and abs(lines[1]["loss"] - 0.3) < 1e-9 and lines[0]["lr"] == 1e-4
    recs = [json.loads(l) for l in sink.read_text().splitlines()]
    assert [r["step"] for r in recs] == [1, 2, 3]
    assert "name" not in recs[0] and abs(recs[2]["loss"] - 0.3) < 1e-9
