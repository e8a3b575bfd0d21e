"""MNISTNet training step (fwd + bwd + Adadelta) on the framework vs plain PyTorch.

    python tools/bench_mnist.py [--batch 64] [--steps 200]

Synthetic 28x28 inputs (no dataset download); the step is the reference's MNIST task step
(tasks.py:337-362 model, Adadelta lr 1.0 as in the reference's mnist recipe).
  framework: the K15 kernels (ops/mnist_ops.py) + the flat parameter store and the one-kernel
             Adadelta (optim/optimizers.py, K14) -- what ``train.py --task mnist`` runs
  torch:     the torch-op network (``logits``: MIOpen convolutions) + torch.optim.Adadelta
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def run(fused, B, steps, warmup):
    from hetseq_amd.models.mnist import MNISTNet

    torch.manual_seed(0)
    model = MNISTNet().cuda().train()
    if fused:
        from types import SimpleNamespace

        from hetseq_amd.optim.optimizers import _Adadelta
        from hetseq_amd.runtime.flat import FlatParamStore

        store = FlatParamStore(model)
        opt = _Adadelta(SimpleNamespace(lr=[1.0], adadelta_rho=0.9, adadelta_eps=1e-6, dadelta_weight_decay=0.0),
                        model.parameters(), store)
    else:
        opt = torch.optim.Adadelta(model.parameters(), lr=1.0)
    x = torch.randn(B, 1, 28, 28, device="cuda")
    t = torch.randint(0, 10, (B,), device="cuda")

    def step():
        if fused:
            opt.zero_grad()
        else:
            opt.zero_grad(set_to_none=True)
        if fused:
            loss = model(x, t)
        else:
            loss = F.nll_loss(F.log_softmax(model.logits(x), dim=1), t)
        loss.backward()
        opt.step()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    for B in sorted({a.batch, 64, 256, 1024}):
        ms_f = run(True, B, a.steps, a.warmup)
        ms_t = run(False, B, a.steps, a.warmup)
        print(json.dumps({"batch": B, "fused_ms": round(ms_f, 4), "torch_ms": round(ms_t, 4),
                          "speedup": round(ms_t / ms_f, 3)}), flush=True)


if __name__ == "__main__":
    main()
