#!/usr/bin/env python3
"""Do the parallel branches of a captured HIP graph run concurrently on replay?

    python tools/graph_branches.py [--us 300] [--side torch|native]

Two spin kernels (the collective stand-in of csrc/kernels/comm_emul.hip: `channels` workgroups that
hold for a fixed wall-clock time) are forked onto two streams and joined -- eagerly, then captured
into a torch.cuda.CUDAGraph and replayed.  Concurrent branches take ~1x the spin time, serialised ones
~2x.  Run once per runtime setting (e.g. DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 / 1) as separate processes.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops._C import hip, stream_handle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--us", type=float, default=300.0)
    ap.add_argument("--side", choices=("torch", "native"), default="torch")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    src = torch.zeros(1 << 20, device=dev)
    scr = torch.zeros(1 << 20, device=dev)
    main_s = torch.cuda.Stream()
    if a.side == "native":
        from hetseq_amd.runtime import streams

        side = streams.side(dev)
    else:
        side = torch.cuda.Stream()

    def spin():
        hip().comm_emulation(src.data_ptr(), 4 << 20, scr.data_ptr(), 4 << 20, 0, 16, int(a.us * 1000), stream_handle())

    def body():
        side.wait_stream(torch.cuda.current_stream())
        spin()
        with torch.cuda.stream(side):
            spin()
        torch.cuda.current_stream().wait_stream(side)

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1000.0 / a.reps

    with torch.cuda.stream(main_s):
        t_eager = timed(body)
        g = torch.cuda.CUDAGraph()
        body()  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=main_s):
            body()
        t_graph = timed(g.replay)
    print(json.dumps({"spin_us": a.us, "side": a.side, "eager_us": round(t_eager, 1), "graph_us": round(t_graph, 1),
                      "packet_capture": os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "(default)")}))


if __name__ == "__main__":
    main()
