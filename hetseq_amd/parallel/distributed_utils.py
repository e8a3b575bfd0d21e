"""Process-group runtime (reference: distributed_utils.py:11-131).

Same entry points: ``distributed_init``, ``is_master``, ``suppress_output``,
``get_rank``/``get_world_size``/``get_default_group``, ``all_reduce`` and
``all_gather_list``.  Differences:

* backend ``nccl`` is RCCL over xGMI on ROCm; ``gloo`` drives CPU runs.  The
  init method may be ``tcp://``, ``file://`` or ``env://``.
* every collective is device-agnostic (the reference hard-codes
  ``torch.cuda.*Tensor``, Q21), so the CPU/gloo path works end to end.
* the warm-up all-reduce also builds the RCCL communicator; a collective
  timeout is configurable (``--collective-timeout``).
* ``all_gather_list`` uses a real all-gather of length-prefixed pickles
  instead of summing a zero-padded buffer.
"""
from __future__ import annotations

import builtins
import datetime
import os
import pickle
import socket
import warnings

import torch
import torch.distributed as dist


def _device_for_backend():
    if dist.get_backend() == "nccl" and torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def distributed_init(args):
    if args.distributed_world_size == 1:
        raise ValueError("Cannot initialize distributed with distributed_world_size=1")
    if dist.is_initialized():
        warnings.warn("Distributed is already initialized, cannot initialize twice!")
    else:
        backend = args.distributed_backend
        if backend == "nccl" and (not torch.cuda.is_available() or getattr(args, "cpu", False)):
            backend = "gloo"  # CPU runs: RCCL needs a GPU
            args.distributed_backend = backend
        print("| distributed init (rank {}): {}".format(args.distributed_rank, args.distributed_init_method), flush=True)
        kw = {}
        if args.distributed_init_method and args.distributed_init_method.startswith("env://"):
            kw = {}
        else:
            kw = dict(world_size=args.distributed_world_size, rank=args.distributed_rank)
        if torch.cuda.is_available() and backend == "nccl":
            from hetseq_amd.runtime import streams

            # the engine's streams take their hardware queues before RCCL creates its streams
            streams.reserve(torch.device("cuda", torch.cuda.current_device()))
        apply_comm_channels(args)
        timeout = datetime.timedelta(seconds=float(getattr(args, "collective_timeout", 1800.0)))
        if backend == "nccl" and torch.cuda.is_available():
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, init_method=args.distributed_init_method, timeout=timeout, **kw)
        print("| initialized host {} as rank {}".format(socket.gethostname(), dist.get_rank()), flush=True)
        # warm-up collective: creates the RCCL communicator / gloo pairs
        dist.all_reduce(torch.zeros(1, device=_device_for_backend()))
        suppress_output(dist.get_rank() == 0)
    args.distributed_rank = dist.get_rank()
    print("| actual rank {}".format(args.distributed_rank))
    return args.distributed_rank


def apply_comm_channels(args):
    """``--comm-channels N``: cap RCCL's channels (one workgroup each, resident on a CU for a
    collective's whole duration, beside the backward's GEMM blocks) before any communicator
    exists.  The value comes from the one-GPU emulation sweep (profiles/r4_dp_emulation.md);
    an NCCL_MAX_NCHANNELS already in the environment wins."""
    n = getattr(args, "comm_channels", None)
    if n and "NCCL_MAX_NCHANNELS" not in os.environ:
        os.environ["NCCL_MAX_NCHANNELS"] = str(int(n))


def shutdown(controller=None):
    """End of a distributed run: every rank reaches a barrier before any rank tears its process
    group down -- a rank that exits while a peer's gloo pair is still reading from it aborts that
    peer ("terminate called without an active exception", seen in the 8-rank CPU rehearsal) -- then
    the native engine and the process group are closed."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    dist.barrier()
    comm = getattr(getattr(controller, "model", None), "comm", None)
    if comm is not None:
        comm.close()
    dist.destroy_process_group()


def is_master(args):
    return args.distributed_rank == 0


_ORIG_PRINT = builtins.print


def suppress_output(is_master):
    """Suppress printing on non-master ranks. Force printing with ``force=True``."""

    def print(*args, **kwargs):
        force = kwargs.pop("force", False)
        if is_master or force:
            _ORIG_PRINT(*args, **kwargs)

    builtins.print = print


def restore_output():
    builtins.print = _ORIG_PRINT


def get_rank():
    return dist.get_rank() if dist.is_initialized() else 0


def get_world_size():
    return dist.get_world_size() if dist.is_initialized() else 1


def get_default_group():
    return dist.group.WORLD


def all_reduce(tensor, group=None):
    if group is None:
        group = get_default_group()
    return dist.all_reduce(tensor, group=group)


def all_gather_list(data, group=None, max_size=16384):
    """Gathers arbitrary picklable data from all ranks into a list (rank order)."""
    world_size = get_world_size()
    if world_size == 1:
        return [data]
    enc = pickle.dumps(data)
    if len(enc) + 4 > max_size:
        raise ValueError("encoded data exceeds max_size: {}".format(len(enc) + 4))
    dev = _device_for_backend()
    buf = torch.zeros(max_size, dtype=torch.uint8)
    buf[:4] = torch.tensor(list(len(enc).to_bytes(4, "little")), dtype=torch.uint8)
    buf[4 : 4 + len(enc)] = torch.frombuffer(bytearray(enc), dtype=torch.uint8)
    buf = buf.to(dev)
    out = torch.empty(world_size * max_size, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.cpu().numpy()
    result = []
    try:
        for i in range(world_size):
            chunk = out[i * max_size : (i + 1) * max_size]
            n = int.from_bytes(bytes(chunk[:4]), "little")
            result.append(pickle.loads(bytes(chunk[4 : 4 + n])))
        return result
    except pickle.UnpicklingError:
        raise Exception(
            "Unable to unpickle data from other workers. all_gather_list requires all "
            "workers to enter the function together, so this error usually indicates "
            "that the workers have fallen out of sync somehow."
        )


def local_device_id(args, local_index):
    """Local process index -> HIP device id (reference: train.py:190; Q24 fix)."""
    return int(local_index) + int(getattr(args, "device_id_offset", 0) or 0)


def env_rank_info():
    """RANK/LOCAL_RANK/WORLD_SIZE from torchrun-style environments (or None)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        return (int(os.environ["RANK"]), int(os.environ.get("LOCAL_RANK", 0)), int(os.environ["WORLD_SIZE"]))
    return None
