"""Weight-gradient layout study: dW = dy^T x on the split-bf16 engine.

Today's wgrad reads both operands mn-contiguous (TA=1, TB=0: 8-wave kernel, register
transpose while staging, ~50% LDS write conflicts in the PMC profile).  Alternative:
transpose dy and x to k-contiguous copies first and run the NT kernel (TA=0, TB=1,
conflict-free k-contiguous staging).  Prints per-shape times of both, the transpose
cost, and the best split-K of each, for the BERT-base call sites (T = 4096).

    python tools/bench_wgrad_layout.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hetseq_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    torch.manual_seed(0)
    T = int(os.environ.get("T", 4096))
    rows = []
    for N, K in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
        dy = torch.randn(T, N, device="cuda")
        x = torch.randn(T, K, device="cuda")
        out = torch.empty(N, K, device="cuda")
        ref = (dy.double().t() @ x.double()).float()
        best_tn = min((timeit(lambda: G._hip_gemm(dy, x, True, False, out, ksplit=ks)), ks) for ks in (0, 1, 2, 4))
        G._hip_gemm(dy, x, True, False, out, ksplit=best_tn[1])
        err_tn = ((out - ref).abs().max() / ref.abs().max()).item()
        dyT = dy.t().contiguous()
        xT = x.t().contiguous()
        best_nt = min((timeit(lambda: G._hip_gemm(dyT, xT, False, True, out, ksplit=ks)), ks) for ks in (0, 1, 2, 4))
        G._hip_gemm(dyT, xT, False, True, out, ksplit=best_nt[1])
        err_nt = ((out - ref).abs().max() / ref.abs().max()).item()
        t_tr = timeit(lambda: (dyT.copy_(dy.t()), xT.copy_(x.t())))
        flop = 2.0 * T * N * K
        rows.append(dict(N=N, K=K, tn_us=round(best_tn[0], 1), tn_ks=best_tn[1], nt_us=round(best_nt[0], 1),
                         nt_ks=best_nt[1], transpose_us=round(t_tr, 1),
                         tn_tfs=round(flop / best_tn[0] / 1e6, 1), nt_tfs=round(flop / best_nt[0] / 1e6, 1),
                         err_tn=err_tn, err_nt=err_nt))
        print(json.dumps(rows[-1]), flush=True)
    tn = sum(r["tn_us"] for r in rows)
    nt = sum(r["nt_us"] + r["transpose_us"] for r in rows)
    print(json.dumps({"per_layer_tn_us": round(tn, 1), "per_layer_nt_plus_transpose_us": round(nt, 1)}))


if __name__ == "__main__":
    main()
