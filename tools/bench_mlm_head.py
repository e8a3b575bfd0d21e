"""Micro-benchmark of the masked-LM decoder GEMMs (bf16 mode): [cap,H] x [V,H]^T.

Compares the plain library calls with split-K / bf16-operand variants:
  dt2   = dlogits[cap,V] @ Wd[V,H]          (K = V = 30522, tiny output -> split-K)
  dWdec = dlogits^T @ t2 -> fp32 [V,H]      (fp32 GEMM today vs bf16 operands + fp32 C)
Usage: python tools/bench_mlm_head.py
"""
import torch


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import os, sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from hetseq_amd.runtime import gemm_tuning

    gemm_tuning.enable("bf16", tune_missing=False)  # the committed tables, like the trainer
    cap, V, H = 640, 30522, 768
    dev = "cuda"
    dl = torch.randn(cap, V, device=dev) * 0.01
    dlb = dl.to(torch.bfloat16)
    Wd = (torch.randn(V, H, device=dev) * 0.02).to(torch.bfloat16)
    t2 = torch.randn(cap, H, device=dev).to(torch.bfloat16)
    ref = dl @ Wd.float()

    def plain():
        return torch.mm(dlb, Wd)

    def splitk(s):
        kc = V // s
        A = dlb.as_strided((s, cap, kc), (kc, V, 1))
        B = Wd.as_strided((s, kc, H), (kc * H, H, 1))
        part = torch.ops.aten.bmm.dtype(A, B, torch.float32)
        out = part.sum(0)
        if kc * s < V:
            out = torch.ops.aten.addmm.dtype(out, dlb[:, kc * s:], Wd[kc * s:], torch.float32)
        return out.to(torch.bfloat16)

    print(f"dt2 plain bf16    {bench(plain):8.1f} us  err {(plain().float() - ref).abs().max().item():.3e}")
    for s in (4, 6, 8, 12, 16):
        f = lambda s=s: splitk(s)
        print(f"dt2 split-K {s:2d}    {bench(f):8.1f} us  err {(f().float() - ref).abs().max().item():.3e}")

    gw = torch.zeros(V, H, device=dev)
    dlf, t2f = dlb.float(), t2.float()

    def wg_fp32():
        gw.addmm_(dlf.t(), t2f)

    def wg_bf16():
        torch.ops.aten.addmm.dtype_out(gw, dlb.t(), t2, torch.float32, beta=1.0, out=gw)

    print(f"dWdec fp32 ops    {bench(wg_fp32):8.1f} us")
    print(f"dWdec bf16 ops    {bench(wg_bf16):8.1f} us")
    logits = torch.empty(cap, V, device=dev)
    bd = torch.zeros(V, device=dev)

    def fwd():
        torch.ops.aten.mm.dtype_out(t2, Wd.t(), torch.float32, out=logits)
        logits.add_(bd)

    print(f"logits fwd        {bench(fwd):8.1f} us")


if __name__ == "__main__":
    main()
