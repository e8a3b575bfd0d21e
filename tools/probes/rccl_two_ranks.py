"""Probe: can two RCCL ranks share the one GPU of a gpurun box?

If RCCL accepts it, the native engine's multi-rank path (bucket all-reduce on the comm
stream, broadcast, in-stream stat all-reduce) can be exercised on a single MI355X; if it
refuses ("duplicate GPU"), the probe reports that and exits 0.

    timeout -k 10 120 python3 tools/probes/rccl_two_ranks.py
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    out = {}
    try:
        t = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        out["c10d"] = float(t[0].item())
    except Exception as e:  # noqa: BLE001
        out["c10d"] = "error: %s" % str(e).splitlines()[0][:200]
    try:
        from hetseq_amd.parallel.comm import NativeComm
        c = NativeComm(timeout_s=60.0)
        g = torch.full((3 << 20,), float(rank + 1), device="cuda")
        c.all_reduce_async(g[: 1 << 20])
        c.all_reduce_async(g[1 << 20:])
        c.wait()
        s = torch.tensor([rank + 1.0], device="cuda")
        c.all_reduce(s)
        torch.cuda.synchronize()
        c.check()
        out["native"] = (float(g.min().item()), float(g.max().item()), float(s.item()))
        c.close()
    except Exception as e:  # noqa: BLE001
        out["native"] = "error: %s" % str(e).splitlines()[0][:200]
    q.put((rank, out))
    dist.destroy_process_group()


def main():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, 29611, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, o = q.get(timeout=100)
        res[r] = o
    for p in procs:
        p.join(timeout=20)
    print("two ranks on one GPU:", res)


if __name__ == "__main__":
    main()
