#!/usr/bin/env python3
"""Which part of a data-parallel step breaks HIP-graph capture (1-rank native communicator).

    python tools/graph_probe.py MODE      (MODE: ar | ag | ar_side | ddp | ddp_tables)

Each mode captures one piece into a torch.cuda.CUDAGraph (thread-local capture mode), replays it
twice and prints ``MODE ok`` -- run the modes as separate processes chained with ``&&``.
"""
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    mode = sys.argv[1]
    cuda = torch.device("cuda", 0)
    torch.cuda.set_device(cuda)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port(), world_size=1, rank=0, device_id=cuda)
    from hetseq_amd.parallel.comm import NativeComm
    from hetseq_amd.runtime import streams

    streams.set_enabled(True)
    if mode.startswith("seq"):  # the tables' sequence on plain tensors
        comm = NativeComm(timeout_s=60)
        keys = torch.randint(0, 100, (768,), device=cuda)
        keys_all = torch.empty_like(keys)
        region = torch.ones(4096, device=cuda)
        rows = torch.ones(256, 64, device=cuda)
        rows_all = torch.empty_like(rows)
        side = torch.cuda.Stream()
        comm.all_reduce(region)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            cur = torch.cuda.current_stream()
            keys.add_(0)
            comm.all_gather_async(keys_all, keys, producers=(cur,))
            use_side = mode != "seq_a"
            if use_side:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    comm.wait()  # side after the key gather
                    if mode == "seq_sort":
                        sk, order = torch.sort(keys_all, stable=True)
                    elif mode == "seq_sort_unstable":
                        sk, order = torch.sort(keys_all)
                    elif mode == "seq_b":
                        keys_all.add_(1)
                    else:
                        sk = keys_all + 1
            comm.all_reduce_async(region, producers=(cur, side) if use_side else (cur,))
            rows.mul_(1.0)
            comm.all_gather_async(rows_all, rows, producers=(cur,))
            if use_side:
                cur.wait_stream(side)
            comm.wait()
            rows_all.add_(1.0)
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        comm.check()
        comm.close()
    elif mode in ("ar", "ag", "ar_side"):
        comm = NativeComm(timeout_s=60)
        x = torch.ones(1 << 20, device=cuda)
        out = torch.empty(1 << 20, device=cuda)
        side = torch.cuda.Stream()
        comm.all_reduce(x)  # warm-up outside capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            x.mul_(1.0)
            if mode == "ar":
                comm.all_reduce_async(x)
            elif mode == "ag":
                comm.all_gather_async(out, x)
            else:
                cur = torch.cuda.current_stream()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    x.add_(0.0)
                comm.all_reduce_async(x, producers=(cur, side))
                cur.wait_stream(side)
            comm.wait()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        comm.check()
        comm.close()
    else:
        from hetseq_amd.parallel.ddp import FlatDDP
        from hetseq_amd.runtime.flat import FlatParamStore
        from tests.test_bert_gpu import _batch, _tiny

        model, cfg = _tiny(cuda)
        model.eval()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="native", timeout_s=60,
                      sparse_embedding=model.sparse_embedding() if mode == "ddp_tables" else None)
        batch = list(_batch(cuda, 4, 64, cfg.vocab_size))
        for _ in range(2):
            store.grad.zero_()
            net(*batch).backward()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            store.grad.zero_()
            net(*batch).backward()
        g.replay()
        g.replay()
        torch.cuda.synchronize()
        net.comm.check()
        net.comm.close()
    print(mode, "ok", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
