"""The h3p GEMM's epilogues on the BERT-base FFN shapes, alone (interleaved rounds, one process):
the FFN-in forward (M 2048 half batch / 4096, N 3072, K 768) plain, +bias, and GELU writing the
pre-activation (aux) and the result's planes; the FFN-out data gradient (M 4096, N 3072, K 768) plain
and through dGELU writing planes and the bias-gradient column partials.

    python tools/bench_h3p_epi.py [--rounds 3]"""
import argparse
import json
import os
import sys

# HS_AB_ROOT: a copy of the package built from another tree (old-vs-new A/B of a kernel change)
sys.path.insert(0, os.environ.get("HS_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import h3p  # noqa: E402


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    H, F = 768, 3072
    for M in (2048, 4096):
        x = h3p.split(torch.randn(M, H, device=dev))
        w1 = h3p.split(torch.randn(F, H, device=dev) * 0.05)
        bi = torch.randn(F, device=dev) * 0.1
        out = torch.empty(M, F, device=dev)
        pre = torch.empty(M, F, device=dev)
        yp = h3p.empty(M, F, dev)
        dy = h3p.split(torch.randn(M, H, device=dev))
        w2 = h3p.split(torch.randn(H, F, device=dev) * 0.05)
        part = torch.empty(M // 128, F, device=dev)
        db = torch.zeros(F, device=dev)
        runs = {
            "fwd plain": lambda: h3p.gemm(x, w1, 0, 1, out=out),
            "fwd bias": lambda: h3p.gemm(x, w1, 0, 1, out=out, bias=bi, epi=h3p.EPI_BIAS),
            "fwd gelu+planes": lambda: h3p.gemm(x, w1, 0, 1, out=None, bias=bi, epi=h3p.EPI_GELU, aux=pre,
                                                planes_out=yp),
            "dgrad plain": lambda: h3p.gemm(dy, w2, 0, 0, out=out),
            "dgrad dgelu+planes": lambda: h3p.gemm(dy, w2, 0, 0, out=None, bias=bi, epi=h3p.EPI_DGELU, aux=pre,
                                                   part=part, colsum=db, colsum_acc=True, planes_out=yp),
        }
        best = {}
        for _ in range(a.rounds):
            for k, fn in runs.items():
                best[k] = min(best.get(k, 1e9), timeit(fn))
        flop = 3 * 2.0 * M * F * H
        print(json.dumps({"M": M, **{k: [round(v, 1), round(flop / (v * 1e-6) / 1e12)] for k, v in best.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
