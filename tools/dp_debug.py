"""Debug: which gradient buckets differ across 2 ranks after one fused backward (gloo, 1 GPU)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch, torch.distributed as dist
rank = int(sys.argv[1]); port = sys.argv[2]
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:" + port, world_size=2, rank=rank)
torch.cuda.set_device(0)
from hetseq_amd.models.bert import BertConfig, BertForPreTraining
from hetseq_amd.runtime.flat import FlatParamStore
from hetseq_amd.parallel.ddp import FlatDDP
from hetseq_amd.runtime import rng
torch.manual_seed(0)
cfg = BertConfig(1000, hidden_size=256, num_hidden_layers=2, num_attention_heads=4, intermediate_size=1024)
m = BertForPreTraining(cfg).cuda()
store = FlatParamStore(m); m.attach_store(store, torch.float32); m.max_predictions_per_seq = 8
ddp = FlatDDP(m, store, bucket_cap_mb=1)
names = {id(p): n for n, p in m.named_parameters()}
orig_launch = ddp._launch
def launch(b):
    print("rank%d launch bucket %d (%d params: %s..)" % (rank, b, len(ddp.buckets[b]), names[id(ddp.buckets[b][0])]), flush=True)
    orig_launch(b)
ddp._launch = launch
g = torch.Generator().manual_seed(rank)
ids = torch.randint(0, 1000, (8, 64), generator=g).cuda()
lab = torch.full((8, 64), -1, dtype=torch.long); lab[:, 5:10] = 7; lab = lab.cuda()
nsp = torch.zeros(8, dtype=torch.long).cuda()
rng.set_seed(5)
store.zero_grad()
loss = ddp(ids, torch.zeros_like(ids), torch.ones_like(ids), lab, nsp)
loss.backward()
torch.cuda.synchronize()
gcpu = store.grad.cpu()
outs = [torch.zeros_like(gcpu) for _ in range(2)]
dist.all_gather(outs, gcpu)
if rank == 0:
    for b, (lo, hi) in enumerate(ddp.ranges):
        d = (outs[0][lo:hi] - outs[1][lo:hi]).abs().max().item()
        if d > 0:
            for p in ddp.buckets[b]:
                o = store.offset(p); n = p.numel()
                dd = (outs[0][o:o+n] - outs[1][o:o+n]).abs().max().item()
                print("  bucket", b, names[id(p)], "diff %.3e" % dd, "norm %.3e" % outs[0][o:o+n].norm().item(), flush=True)
    print("max diff", (outs[0] - outs[1]).abs().max().item())
dist.destroy_process_group()
