#!/usr/bin/env python3
"""RCCL all-reduce bandwidth vs message size over xGMI.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/allreduce_bench.py

For each size (default: 1 MB .. 512 MB, which brackets the 25 MB bucket and the 440 MB
BERT-base gradient) rank 0 prints time, algorithm bandwidth (bytes / t) and bus bandwidth
(2 (W-1)/W * bytes / t, the per-GPU link traffic of a ring) -- the numbers to size
--bucket-cap-mb against.  Also times the FlatDDP bucket pattern: one flat buffer
reduced as consecutive slices of the bucket size.
"""
import argparse
import os
import time

import torch
import torch.distributed as dist


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,25,64,128,256,440,512")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    a = ap.parse_args()
    rank, world, local = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    for mb in [float(x) for x in a.sizes_mb.split(",")]:
        n = int(mb * 2 ** 20) // 4
        x = torch.ones(n, device="cuda")
        t = timed(lambda: dist.all_reduce(x), a.iters)
        if rank == 0:
            algbw = n * 4 / t / 1e9
            print("allreduce %8.1f MB  %8.3f ms  algbw %7.1f GB/s  busbw %7.1f GB/s" %
                  (mb, t * 1e3, algbw, algbw * 2 * (world - 1) / world), flush=True)
    # the FlatDDP pattern: 440 MB of fp32 gradients as async bucket slices
    n = 110_106_428
    flat = torch.ones(n, device="cuda")
    step = int(a.bucket_mb * 2 ** 20) // 4

    def buckets():
        works = [dist.all_reduce(flat[o:o + step], async_op=True) for o in range(0, n, step)]
        for w in works:
            w.wait()

    t = timed(buckets, max(3, a.iters // 4))
    if rank == 0:
        print("flat 440 MB in %.0f MB buckets: %.3f ms (%d buckets)" % (a.bucket_mb, t * 1e3, (n + step - 1) // step))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
