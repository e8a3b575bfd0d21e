#!/usr/bin/env python3
"""|max| passes of the h3 engine over BERT-base-sized data: amax_seg over the 110 M-float flat store
(per-weight segments) at several block chunk sizes, and amax over one 12.6 MB activation.

    python tools/bench_amax.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402
from hetseq_amd.ops._C import hip, stream_handle  # noqa: E402


def timeit(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    flat = torch.randn(110106432, device="cuda")
    # 50 weight-like segments: 12 layers x (2304x768, 768x768, 3072x768, 768x3072) + two head matrices
    sizes = [2304 * 768, 768 * 768, 3072 * 768, 768 * 3072] * 12 + [768 * 768, 30522 * 768]
    ts, off = [], 0
    for n in sizes:
        ts.append(flat[off:off + n])
        off += (n + 63) // 64 * 64
    out = torch.zeros(len(ts) * G.SLOT_FLOATS, device="cuda")
    for chunk in (16384, 8192, 4096, 2048):
        G._SEG_CHUNK4 = chunk
        G._SEG_TABLES.clear()
        base, tab, nblk = G._seg_table(ts)
        t = []
        for _ in range(3):
            t.append(timeit(lambda: hip().amax_seg(base, tab.data_ptr(), nblk, out.data_ptr(), stream_handle())))
        t = statistics.median(t)
        print("amax_seg chunk %5d float4 (%d blocks): %.1f us  %.2f TB/s" % (chunk, nblk, t, 4 * off / t / 1e6))
    x = torch.randn(4096 * 768, device="cuda")
    slot = torch.zeros(G.SLOT_FLOATS, device="cuda")
    t = timeit(lambda: hip().amax(x.data_ptr(), x.numel(), slot.data_ptr(), 0, stream_handle()))
    print("amax 12.6 MB: %.1f us" % t)


if __name__ == "__main__":
    main()
