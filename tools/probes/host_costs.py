"""Host cost of the launch primitives (us per call): stream fork (event record + wait), a small kernel
launch through the extension, torch.cuda.Event record / wait, a layer-program forward / backward call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from hetseq_amd.ops._C import hip, stream_handle  # noqa: E402
from hetseq_amd.runtime import streams  # noqa: E402


def per_call(fn, n=2000):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return round(dt, 2)


dev = torch.device("cuda", 0)
side = streams.side(dev).cuda_stream
cur = stream_handle()
x = torch.zeros(1 << 16, device=dev)
part = torch.zeros(64, 1024, device=dev)
out = torch.zeros(1024, device=dev)
ev = torch.cuda.Event()
res = {
    "stream_wait (record+wait)": per_call(lambda: hip().stream_wait(side, cur)),
    "colsum launch (64x1024)": per_call(lambda: hip().colsum(0, x.data_ptr(), 0, 0, 0, part.data_ptr(), out.data_ptr(),
                                                             64, 1024, 1, cur)),
    "torch Event record": per_call(lambda: ev.record()),
    "torch Event wait": per_call(lambda: torch.cuda.current_stream().wait_event(ev)),
    "torch.empty 1 MB": per_call(lambda: torch.empty(1 << 18, device=dev)),
    "stream_handle()": per_call(stream_handle),
}
for k, v in res.items():
    print("%-28s %8.2f us" % (k, v))
