"""Diagnostic: replicate __graft_entry__.smoke step by step with prints (HIP launch failures)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

print("env", {k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith("HIP") or k.startswith("HSA")})
print("avail", torch.cuda.is_available(), "count", torch.cuda.device_count(), "cur", torch.cuda.current_device())
from hetseq_amd.ops import bert_ops  # noqa: E402
from hetseq_amd.ops._C import hip  # noqa: E402

h = hip()
x = torch.randn(64, 256, device="cuda")
g = torch.ones(256, device="cuda")
b = torch.zeros(256, device="cuda")
for step in ("layer_norm", "smoke"):
    try:
        if step == "layer_norm":
            y = bert_ops.layer_norm(x, g, b)
            torch.cuda.synchronize()
            print("layer_norm ok", float(y.abs().sum()))
        else:
            import __graft_entry__ as ge

            ge.smoke()
    except Exception as e:
        print(step, "FAIL", repr(e))
