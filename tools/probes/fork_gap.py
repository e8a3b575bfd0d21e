#!/usr/bin/env python3
"""GPU cost of the backward's stream forks: dependent small kernels on one stream, with and without an
event record (+ a side-stream wait on it) between them.  The stream is first held by a sleep kernel so
the host enqueues everything ahead of the GPU (host launch cost does not show).

    python tools/probes/fork_gap.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from hetseq_amd.ops._C import hip, stream_handle  # noqa: E402
from hetseq_amd.runtime import streams  # noqa: E402


def run(mode, n=200):
    dev = torch.device("cuda", 0)
    x = torch.zeros(4096, device=dev)
    side = streams.side(dev)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)  # ~0.1 s: the host enqueues the rest meanwhile
    s.record()
    for _ in range(n):
        x.add_(1.0)
        if mode == "record":
            hip().stream_wait(side.cuda_stream, stream_handle())  # record on compute, side waits
        elif mode == "roundtrip":
            hip().stream_wait(side.cuda_stream, stream_handle())
            hip().stream_wait(stream_handle(), side.cuda_stream)  # and compute waits for side
        elif mode == "side_kernel":
            streams.run(dev, lambda: x.mul(1.0))  # fork + a kernel on the side stream
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / n


if __name__ == "__main__":
    streams.reserve(torch.device("cuda", 0))
    for flags in (0, 1, 2):
        hip().set_stream_wait_flags(flags)
        for m in ("plain", "record", "roundtrip"):
            ts = sorted(run(m) for _ in range(5))
            print("flags %d %-12s %.2f us per step (median of 5)" % (flags, m, ts[2]))
    hip().set_stream_wait_flags(0)
