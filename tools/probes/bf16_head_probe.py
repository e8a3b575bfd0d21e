"""bf16 MLM head: per-parameter gradient differences of the padded plane-kernel decoder and the library
decoder against an fp32 model's gradients (diagnostic for tests/test_bert_gpu.py)."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))

import torch  # noqa: E402

import hetseq_amd.models.bert as MB  # noqa: E402
from hetseq_amd.runtime.flat import FlatParamStore  # noqa: E402
from test_bert_gpu import _batch, _tiny  # noqa: E402

cuda = torch.device("cuda", 0)
model, cfg = _tiny(cuda)
model.eval()
model.max_predictions_per_seq = 32
ref, m32, again = copy.deepcopy(model), copy.deepcopy(model), copy.deepcopy(model)
stores = []
for m in (model, ref, again):
    st = FlatParamStore(m, shadow_dtype=torch.bfloat16)
    m.attach_store(st, torch.bfloat16)
    stores.append(st)
s32 = FlatParamStore(m32)
m32.attach_store(s32, torch.float32)
batch = _batch(cuda, 4, 128, cfg.vocab_size)
MB.HEAD_BF16_PAD = True
l1 = model(*batch)
l1.backward()
MB.HEAD_BF16_PAD = False
l2 = ref(*batch)
l2.backward()
l3 = m32(*batch)
l3.backward()
MB.HEAD_BF16_PAD = True
l4 = again(*batch)
l4.backward()
print("loss pad %.6f lib %.6f fp32 %.6f pad-again %.6f" % (l1.item(), l2.item(), l3.item(), l4.item()))
for (n, p1), (_, p2), (_, p3), (_, p4) in zip(model.named_parameters(), ref.named_parameters(), m32.named_parameters(),
                                              again.named_parameters()):
    d = stores[2].grad[stores[2].offset(p4):][:p4.numel()].double()
    a = stores[0].grad[stores[0].offset(p1):][:p1.numel()].double()
    b = stores[1].grad[stores[1].offset(p2):][:p2.numel()].double()
    c = s32.grad[s32.offset(p3):][:p3.numel()].double()
    sc = c.abs().max().item() + 1e-30
    print("%-55s |g| %.3e  pad-fp32 %.3e  lib-fp32 %.3e  again-fp32 %.3e  pad-lib %.3e" % (
        n, sc, (a - c).abs().max().item() / sc, (b - c).abs().max().item() / sc, (d - c).abs().max().item() / sc,
        (a - b).abs().max().item() / sc))
