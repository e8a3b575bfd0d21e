#!/usr/bin/env python3
"""fp32 Adam pass (optim.hip adam_flat_kernel) launch shapes over BERT-base's 110 M parameters:
grid cap x float4 groups per thread x streaming accesses; prints us and effective TB/s (7 streams).

    python tools/bench_adam.py [--n 110106428]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops._C import hip, stream_handle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=110106432)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n = a.n
    p, g, m, v = (torch.randn(n, device="cuda") * 0.01 for _ in range(4))
    v.abs_()
    gm = torch.ones(1, device="cuda")

    def run():
        hip().adam_flat(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), 0, n, gm.data_ptr(), 1e-4, 0.9, 0.999,
                        1e-6, 0.01, 1e-4, stream_handle())

    cfgs = [(8192, 2, 1), (16384, 2, 1), (32768, 2, 1), (65536, 2, 1), (53760, 2, 1), (131072, 1, 1),
            (65536, 4, 1), (65536, 2, 0)]
    res = {c: [] for c in cfgs}
    for _ in range(3):  # interleaved rounds
        for c in cfgs:
            hip().set_adam_config(*c)
            run()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                run()
            e.record()
            e.synchronize()
            res[c].append(s.elapsed_time(e) * 1000.0 / a.reps)
    hip().set_adam_config(65536, 2, 1)
    part = torch.zeros(1024, dtype=torch.float64, device="cuda")
    out = torch.zeros(4, device="cuda")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    hip().grad_norm(g.data_ptr(), n, part.data_ptr(), gm.data_ptr(), 1.0, out.data_ptr(), stream_handle())
    s.record()
    for _ in range(a.reps):
        hip().grad_norm(g.data_ptr(), n, part.data_ptr(), gm.data_ptr(), 1.0, out.data_ptr(), stream_handle())
    e.record()
    e.synchronize()
    t = s.elapsed_time(e) * 1000.0 / a.reps
    print("grad norm (sumsq + finalize): %.1f us  %.2f TB/s" % (t, 4 * n / t / 1e6))
    for c, ts in res.items():
        t = statistics.median(ts)
        print("grid %5d unroll %d nt %d: %7.1f us  %.2f TB/s" % (c[0], c[1], c[2], t, 7 * 4 * n / t / 1e6))


if __name__ == "__main__":
    main()
