"""Headline benchmark: avg sec/step of BERT-base phase-1 pre-training.

Config (BASELINE.json): BERT-base (110,106,428 params, random init),
seq_len 128, 32 sequences per GPU per step (update-freq 1), synthetic
NVIDIA-format HDF5 shards read through the native loader, fused Adam,
--fast-stat-sync (as in every documented reference run), weak scaling.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp32|bf16] [--hetero 2,6]

Launch modes (one process per GPU, RCCL over xGMI):

* ``torchrun --nproc-per-node N bench.py --gpus N`` -- the ranks come from
  RANK / LOCAL_RANK / WORLD_SIZE; a ``--gpus`` that disagrees with WORLD_SIZE is
  an error (exit 2), never a silently smaller run.
* ``python bench.py --gpus N`` (N > 1, no WORLD_SIZE) -- this process becomes a
  launcher: it starts N fresh rank processes (env:// rendezvous on 127.0.0.1),
  never touches the GPU itself, relays their output and exits non-zero if any
  rank fails.
* ``python bench.py --hetero 2,6`` -- the heterogeneous launch of BASELINE.json
  config 4: one launch group per entry (here 2 and 6 GPUs of one node), each
  with its own ``--distributed-gpus`` / first global rank / ``--device-id-offset``,
  joined by a ``tcp://`` rendezvous, exactly like separate ``train.py`` launches
  on two nodes (reference train.py:189-236).

Timed region: K full training steps (data -> H2D -> fwd -> bwd -> bucketed
all-reduce -> stats all-reduce -> clip -> Adam), bracketed by a barrier and
device synchronisation on both sides; the reported time is the MAX over
ranks.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

BASELINE_SEC_PER_STEP = 2.60  # README.md:65, 1 node x 4 GPUs, 32 seq/GPU/step


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (= ranks); default WORLD_SIZE under torchrun, else 1")
    p.add_argument("--hetero", default=None,
                   help="heterogeneous launch groups, e.g. 2,6: one launch per group (tcp:// rendezvous)")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--seq-len", type=int, default=128)
    p.add_argument("--batch", type=int, default=32)
    p.add_argument("--max-pred", type=int, default=20)
    p.add_argument("--update-freq", type=int, default=1)
    p.add_argument("--layers", type=int, default=12)
    p.add_argument("--bucket-cap-mb", type=int, default=25)
    p.add_argument("--no-fused", action="store_true")
    p.add_argument("--gemm", default=None, choices=[None, "hip", "blas"])
    p.add_argument("--profile-phases", action="store_true")
    p.add_argument("--hip-graph", action="store_true", help="replay the captured update as one HIP graph (1 GPU, or data-parallel on the native RCCL engine)")
    p.add_argument("--sync-debug", action="store_true", help="warn (with stack) on every host<->device sync in the timed loop")
    p.add_argument("--host-phases", action="store_true",
                   help="host time per step of each train_step phase (forward, backward, norm, step, ...)")
    p.add_argument("--host-delay-us", type=float, default=0.0,
                   help=argparse.SUPPRESS)  # diagnostic: host sleep before every timed step (the host's slack)
    p.add_argument("--prefill-us", type=float, default=0.0,
                   help=argparse.SUPPRESS)  # diagnostic: a spin kernel of this length right before the timed loop
    # (gives the host a head start: if the step's device gaps are host-caused, they disappear)
    p.add_argument("--host-profile", default=None, help="cProfile the timed loop into this file")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend for N > 1 (nccl = RCCL; gloo only to rehearse several ranks on one GPU)")
    p.add_argument("--comm-engine", default="auto", choices=["auto", "native", "c10d"],
                   help="gradient collectives for N > 1: native RCCL engine (auto with nccl) or torch c10d")
    p.add_argument("--dry-run", type=int, default=None, help=argparse.SUPPRESS)  # launcher test: fail this rank
    # profiling aid: the data-parallel engine (FlatDDP + native RCCL comm stream) on a 1-rank world,
    # so the stream / HW-queue layout of a DP step can be traced on one GPU (profiles/r3_stream_queues.md)
    p.add_argument("--ddp-world1", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--ab", default=None,
                   help="A/B mode (1 GPU): alternate these runtime variants (comma list of " + ",".join(sorted(_AB))
                        + ") in --ab-rounds rounds of --steps steps each, one process, and print each variant's "
                        "median ms per step (interleaving cancels drift in the box's clock / thermal state)")
    p.add_argument("--ab-rounds", type=int, default=6, help=argparse.SUPPRESS)
    p.add_argument("--fp32-gemm", default=None, choices=[None, "h3p", "h3", "x6", "native"],
                   help="fp32 GEMM engine (default: HETSEQ_FP32_GEMM or the built-in default)")
    p.add_argument("--emulate-world", type=int, default=None, metavar="W",
                   help="1 GPU: predict the W-rank data-parallel step -- the DP engine on a 1-rank RCCL world whose "
                        "bucket collectives are replaced by stand-in kernels with W-rank traffic, duration and "
                        "channel footprint (parallel/comm.py set_emulation); the JSON carries comm_emulated: W")
    p.add_argument("--emulate-busbw", type=float, default=400.0, metavar="GB/s",
                   help="bus bandwidth of the emulated ring collectives (per-rank received bytes / time)")
    p.add_argument("--emulate-latency-us", type=float, default=12.0, help="fixed cost per emulated collective")
    p.add_argument("--no-shard-optimizer", action="store_true",
                   help="data parallel: every rank runs the whole Adam update (default: sharded, parallel/zero.py)")
    p.add_argument("--no-sparse-tables", action="store_true",
                   help="data parallel: all-reduce the embedding tables densely in the last bucket (no sparse row exchange)")
    p.add_argument("--comm-channels", type=int, default=None,
                   help="RCCL channel cap (NCCL_MAX_NCHANNELS) of real runs; workgroups per emulated collective "
                        "(default 32 when emulating)")
    p.add_argument("--gemm-choices", default=None,
                   help="JSON of measured GEMM engine choices: loaded if it exists (no measuring in warm-up), "
                        "else written after the run (profiling runs use it to keep tuning out of the trace)")
    return p.parse_args()




def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _groups(b):
    """Launch groups: [(n_ranks, first_global_rank)]."""
    if b.hetero:
        sizes = [int(x) for x in b.hetero.split(",") if x.strip()]
        if not sizes or min(sizes) < 1:
            raise SystemExit("bench.py: bad --hetero %r" % b.hetero)
        out, r = [], 0
        for n in sizes:
            out.append((n, r))
            r += n
        return out
    return [(b.gpus, 0)]


def launch(b):
    """Parent of a self-launched multi-rank run: starts one fresh process per rank, relays their
    output, fails if any rank fails.  This process never initialises the GPU (no torch import)."""
    groups = _groups(b)
    world = sum(n for n, _ in groups)
    port = _free_port()
    procs = []
    for gi, (n, first) in enumerate(groups):
        for i in range(n):
            env = dict(os.environ)
            env.update({"RANK": str(first + i), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                        "MASTER_PORT": str(port), "HETSEQ_BENCH_CHILD": "1"})
            if b.hetero:
                # one launch group = one "node" of the heterogeneous job: local index i inside it,
                # devices from the group's offset, tcp:// rendezvous (reference train.py:213-225)
                env.update({"LOCAL_RANK": str(i), "LOCAL_WORLD_SIZE": str(n), "HETSEQ_GROUP": str(gi),
                            "HETSEQ_GROUP_GPUS": str(n), "HETSEQ_DEVICE_OFFSET": str(first),
                            "HETSEQ_INIT_METHOD": "tcp://127.0.0.1:%d" % port})
            else:
                env.update({"LOCAL_RANK": str(first + i), "LOCAL_WORLD_SIZE": str(world)})
            cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
            procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0 and rc == 0:
                    rc = r
                    print("bench.py: rank process %d exited with %d; stopping the others" % (procs.index(p), r),
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    b = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if b.hetero and b.gpus is not None and b.gpus != sum(n for n, _ in _groups(b)):
        print("bench.py: --gpus %d disagrees with --hetero %s" % (b.gpus, b.hetero), file=sys.stderr)
        return 2
    if env_world is None:
        if b.hetero:
            return launch(b)
        b.gpus = 1 if b.gpus is None else b.gpus
        if b.gpus > 1:
            return launch(b)
    elif b.gpus is not None and b.gpus != int(env_world) and not b.hetero:
        print("bench.py: --gpus %d disagrees with WORLD_SIZE=%s (the launcher started a different number of "
              "ranks); refusing to time a different job" % (b.gpus, env_world), file=sys.stderr)
        return 2
    return run_rank(b)


def run_rank(b):
    if b.dry_run is not None:
        # launcher test hook (tests/test_bench_launch.py): report the rank layout, touch nothing
        rank = int(os.environ.get("RANK", "0"))
        info = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT", "HETSEQ_GROUP",
                                               "HETSEQ_GROUP_GPUS", "HETSEQ_DEVICE_OFFSET", "HETSEQ_INIT_METHOD")}
        sys.stdout.write("DRYRUN " + json.dumps(info) + "\n")  # one write: ranks share the pipe
        sys.stdout.flush()
        return 3 if b.dry_run == rank else 0
    if b.gemm:
        os.environ["HETSEQ_GEMM"] = b.gemm
    if b.fp32_gemm:
        os.environ["HETSEQ_FP32_GEMM"] = b.fp32_gemm
    if b.emulate_world and b.emulate_world > 1:
        if int(os.environ.get("WORLD_SIZE", "1")) != 1:
            print("bench.py: --emulate-world runs on ONE rank", file=sys.stderr)
            return 2
        b.ddp_world1 = True  # the DP engine on a 1-rank world, native RCCL engine, emulated collectives
        b.comm_engine = "native"
    import torch
    import torch.distributed as dist

    from hetseq_amd import options
    from hetseq_amd.controller import Controller
    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.parallel import distributed_utils
    from hetseq_amd.tasks import LanguageModelingTask

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    hetero = os.environ.get("HETSEQ_INIT_METHOD") is not None
    work = tempfile.mkdtemp(prefix="hetseq_bench_r%d_" % rank)
    data_dir = os.path.join(work, "data")
    # every rank writes the SAME shards (same seed) and takes its strided share of the
    # globally shuffled batch list, exactly like training (index randomisation + assignment)
    per_shard = max(256, b.batch * b.update_freq * (b.steps + b.warmup + 2) * world // 2 + 1)
    write_bert_shards(data_dir, num_shards=2, per_shard=per_shard, seq_len=b.seq_len, max_pred=b.max_pred,
                      vocab_size=30522, seed=17, split="train", full_length=False)
    write_vocab(os.path.join(work, "vocab.txt"))
    cfg = write_bert_config(os.path.join(work, "bert_base.json"), num_hidden_layers=b.layers)
    argv = ["--task", "bert", "--data", data_dir, "--dict", os.path.join(work, "vocab.txt"), "--config_file", cfg,
            "--max-sentences", str(b.batch), "--lr", "1e-4", "--warmup-updates", "100", "--weight-decay", "0.01",
            "--fast-stat-sync", "--clip-norm", "25", "--dtype", b.dtype, "--bucket-cap-mb", str(b.bucket_cap_mb),
            "--distributed-world-size", str(world), "--num-workers", "2", "--log-format", "none",
            "--update-freq", str(b.update_freq), "--comm-engine", b.comm_engine]
    if b.no_fused:
        argv.append("--no-fused")
    if b.comm_channels:
        argv += ["--comm-channels", str(b.comm_channels)]
    if b.no_sparse_tables:
        argv.append("--no-sparse-embedding-exchange")
    if b.no_shard_optimizer:
        argv += ["--shard-optimizer", "off"]
    if b.emulate_world and b.emulate_world > 1:
        argv += ["--emulate-world", str(b.emulate_world)]
    if b.hip_graph:
        argv.append("--hip-graph")
    if world > 1:
        argv += ["--distributed-backend", b.dist_backend, "--distributed-rank", str(rank)]
        if hetero:  # this rank's launch group: its GPU count and device offset on the node
            argv += ["--distributed-init-method", os.environ["HETSEQ_INIT_METHOD"],
                     "--distributed-gpus", os.environ["HETSEQ_GROUP_GPUS"],
                     "--device-id-offset", os.environ["HETSEQ_DEVICE_OFFSET"]]
        else:
            argv += ["--distributed-init-method", "env://"]
    args = options.parse_cli(argv)
    args.distributed_rank = rank
    args.force_ddp = bool(b.ddp_world1 and world == 1)
    # local index -> device (group offset for heterogeneous launches); gloo rehearsal: all on GPU 0,
    # but the map the nccl path would use is still computed here and reported (JSON device_map)
    mapped_device = distributed_utils.local_device_id(args, local_rank)
    args.device_id = 0 if b.dist_backend == "gloo" else mapped_device
    torch.cuda.set_device(args.device_id)
    from hetseq_amd.runtime import streams

    streams.reserve(torch.device("cuda", args.device_id))  # hardware queues before RCCL's streams
    if args.force_ddp:
        distributed_utils.apply_comm_channels(args)
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), world_size=1, rank=0,
                                device_id=torch.device("cuda", args.device_id))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        distributed_utils.distributed_init(args)  # the training launcher's own rendezvous + warm-up
        if b.dist_backend == "gloo":
            dist.all_reduce(torch.zeros(1, device="cuda"))  # (touch the device as the nccl path does)
    torch.manual_seed(args.seed)
    task = LanguageModelingTask.setup_task(args)
    model = task.build_model(args)
    nparams = sum(p.numel() for p in model.parameters())
    from hetseq_amd.runtime import gemm_tuning

    gemm_tuning.configure(args)
    ctl = Controller(args, task, model)
    task.load_dataset("train")
    task.prepare_model_for_data(ctl.get_model(), "train")
    epoch_itr = task.get_batch_iterator(task.dataset("train"), max_sentences=b.batch, seed=args.seed, num_shards=world,
                                        shard_id=rank, num_workers=2, epoch=0, device=ctl.device)

    def batches():
        while True:
            itr = epoch_itr.next_epoch_itr(shuffle=True)
            group = []
            for s in itr:
                if s is None or s[0].shape[0] != b.batch:
                    continue
                group.append(s)
                if len(group) == b.update_freq:
                    yield group
                    group = []

    gen = batches()
    if b.gemm_choices and os.path.exists(b.gemm_choices):
        G.load_choices(b.gemm_choices)
    ctl.optimizer  # build optimizer/scheduler (and the DP engine) before timing
    comm_id = _comm_identity(ctl, world, rank)
    emul = None
    if b.emulate_world and b.emulate_world > 1:
        comm = getattr(ctl.model, "comm", None)
        if comm is None:
            print("bench.py: --emulate-world needs the native RCCL engine (%s)"
                  % __import__("hetseq_amd.parallel.comm", fromlist=["LAST_STATUS"]).LAST_STATUS, file=sys.stderr)
            return 2
        emul = {"world": b.emulate_world, "channels": b.comm_channels or 32, "busbw_gbs": b.emulate_busbw,
                "latency_us": b.emulate_latency_us}
        comm.set_emulation(b.emulate_world, emul["channels"], b.emulate_busbw, b.emulate_latency_us)
        _EMUL.update(emul, comm=comm)
    for _ in range(b.warmup):
        ctl.train_step(next(gen))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if b.sync_debug:
        torch.cuda.set_sync_debug_mode("warn")
    prof = None
    if b.host_profile:
        import cProfile

        torch.autograd.set_multithreading_enabled(False)  # backward on this thread, visible to cProfile
        prof = cProfile.Profile()
        prof.enable()
    if b.ab:
        return _ab_run(b, ctl, gen)
    phases = _host_phases(ctl) if b.host_phases else None
    ms0 = torch.cuda.memory_stats()
    if b.prefill_us > 0:
        from hetseq_amd.ops._C import hip as _hip, stream_handle as _sh

        _pf = torch.zeros(1 << 16, device="cuda")
        _hip().comm_emulation(_pf.data_ptr(), _pf.numel() * 4, _pf.data_ptr(), _pf.numel() * 4, 0, 8,
                              int(b.prefill_us * 1000), _sh())
    t0 = time.perf_counter()
    host = 0.0  # host time spent inside train_step (enqueue cost; < ms_per_step means GPU-bound)
    data_wait = 0.0  # host time blocked on the input pipeline
    for _ in range(b.steps):
        d0 = time.perf_counter()
        batch = next(gen)
        if b.host_delay_us > 0:
            time.sleep(b.host_delay_us * 1e-6)
        h0 = time.perf_counter()
        data_wait += h0 - d0
        ctl.train_step(batch)
        host += time.perf_counter() - h0
    if b.sync_debug:
        torch.cuda.set_sync_debug_mode(0)
    if prof is not None:
        prof.disable()
        prof.dump_stats(b.host_profile)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ms1 = torch.cuda.memory_stats()
    # device-level allocator events inside the timed loop (each hipMalloc / hipFree can stall the host)
    alloc_events = {k: ms1.get(k, 0) - ms0.get(k, 0) for k in ("num_device_alloc", "num_device_free",
                                                             "num_alloc_retries", "num_sync_all_streams")}
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    loss = float(ctl.get_meter("train_loss").avg)
    from hetseq_amd.ops import bert_ops

    bert_ops.check_device_errors()
    sec = elapsed / b.steps
    seqs = b.batch * b.update_freq * world
    me = {"rank": rank, "local_rank": local_rank, "group": int(os.environ.get("HETSEQ_GROUP", "0")),
          "device_id": mapped_device, "ran_on": args.device_id}
    device_map = [me]
    if world > 1:  # every rank's computed rank -> device map, in rank order (rank 0 reports it)
        device_map = [None] * world
        dist.all_gather_object(device_map, me)
    if rank == 0 and b.gemm_choices and not os.path.exists(b.gemm_choices):
        G.save_choices(b.gemm_choices)
    if rank == 0:
        from hetseq_amd.parallel import comm as native_comm

        comm_kind = "none" if (world == 1 and not args.force_ddp) else (
            "rccl-native" if getattr(ctl.model, "comm", None) is not None else "c10d-" + b.dist_backend)
        par = "dp%d" % world + (" (hetero %s)" % "+".join(str(n) for n, _ in _groups(b)) if b.hetero else "") + (
            " (DP engine on a 1-rank world)" if args.force_ddp else "") + (
            " emulating dp%d" % emul["world"] if emul else "")
        out = {
            "metric": "avg sec/step, BERT-base seq%d bs=%d/GPU" % (b.seq_len, b.batch),
            "value": round(sec, 6),
            "unit": "s/step",
            "n_gpus": world,
            "steps": b.steps,
            "warmup": b.warmup,
            "ms_per_step": round(sec * 1000, 3),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": round(sec / BASELINE_SEC_PER_STEP, 6),
            "speedup_vs_baseline": round(BASELINE_SEC_PER_STEP / sec, 2),
            "seq_per_s": round(seqs / sec, 1),
            "tokens_per_s": round(seqs * b.seq_len / sec, 1),
            "dtype": b.dtype,
            "data": "synthetic NVIDIA-format HDF5 shards (random tokens), random-init weights",
            "config": {"model": "bert-base-uncased (L12 H768 A12, %d params)" % nparams,
                       "global_batch": seqs, "seq_len": b.seq_len, "per_gpu_batch": b.batch,
                       "update_freq": b.update_freq, "parallelism": par,
                       "fused_kernels": not b.no_fused, "bucket_cap_mb": b.bucket_cap_mb,
                       "hip_graph": bool(getattr(ctl, "_graph", None)), "comm": comm_kind,
                       "comm_fallback_reason": native_comm.LAST_STATUS.get("reason") if world > 1 else None},
            "final_train_loss_logged": round(loss, 5),
            "host_ms_per_step": round(host / b.steps * 1000, 3),
            "data_wait_ms_per_step": round(data_wait / b.steps * 1000, 3),
            "allocator_events": alloc_events,
            "host_phases_ms": ({k: [round(v[0] / b.steps * 1000, 3), round(v[1] * 1000, 3)] for k, v in phases.items()}
                               if phases is not None else None),  # [mean per step, max]
            "gemm_choices": {str(k): v for k, v in list(G.GEMM_CHOICES.items())[:32]},
            "fp32_gemm": G.fp32_mode(),
            "device_map": device_map,
            "rccl_ranks": comm_id[0].get("rccl_count", 1 if world == 1 else None),
            "comm_identity": comm_id,
            "comm_emulated": emul["world"] if emul else None,
            "emulation": emul,
        }
        ddp = ctl.model if hasattr(ctl.model, "comm_log") else None
        if ddp is not None:  # the last step's collectives: count, payload and received bytes, exposed tail
            out["dp_collectives"] = {"n": len(ddp.comm_log), "payload_mb": round(sum(x[1] for x in ddp.comm_log) / 2**20, 2),
                                     "received_mb": round(sum(x[3] for x in ddp.comm_log) / 2**20, 2),
                                     "tail_received_mb": round(ddp.tail_bytes() / 2**20, 2),
                                     "buckets": len(ddp.buckets), "sparse_tables": ddp.tables is not None}
        sys.stdout.write(json.dumps(out) + "\n")  # one write: other ranks may share this pipe
        sys.stdout.flush()
    if world > 1 or args.force_ddp:
        dist.barrier()
        if getattr(ctl.model, "comm", None) is not None:
            ctl.model.comm.close()
        dist.destroy_process_group()
    return 0


_EMUL: dict = {}  # the emulation in force (bench.py --emulate-world), for the --ab channel variants


def _set_emul_channels(n):
    _EMUL["channels"] = n
    _EMUL["comm"].set_emulation(_EMUL["world"], n, _EMUL["busbw_gbs"], _EMUL["latency_us"])


def _set_emul_busbw(gbs):
    _EMUL["busbw_gbs"] = gbs
    _EMUL["comm"].set_emulation(_EMUL["world"], _EMUL["channels"], gbs, _EMUL["latency_us"])


def _set_ln_partials(on):
    from hetseq_amd.ops import bert_ops

    bert_ops._LN_PARTIALS = on


def _set_side_ks(big, small):
    from hetseq_amd.runtime import streams

    streams.SIDE_KSPLIT, streams.SIDE_KSPLIT_SMALL = big, small


def _set_flag(mod, name, v):
    import importlib

    setattr(importlib.import_module(mod), name, v)


def _set_head_engine(engine):
    from hetseq_amd.ops import gemm as G

    for k in list(G.GEMM_CHOICES):
        if len(k) == 7 and 640 in k[:3] and 30522 not in k[:3]:  # (M, N, K, ta, tb, epi, beta)
            c = G.GEMM_CHOICES[k]
            G.GEMM_CHOICES[k] = (engine,) + tuple(c[1:])


def _set_decoder_dgrad_ks(ks):
    from hetseq_amd.ops import gemm as G

    for k, c in list(G.GEMM_CHOICES.items()):
        if len(k) == 4 and k[3] == "decoder_dgrad" and c[0] == "hip":
            G.GEMM_CHOICES[k] = tuple(c[:3]) + (ks,)


def _set_site_ks(key, ks):
    from hetseq_amd.ops import gemm as G

    c = G.GEMM_CHOICES.get(key)
    if c is not None:
        G.GEMM_CHOICES[key] = tuple(c[:3]) + (ks,)


# runtime variants for --ab (switches that take effect on the next step without a rebuild)
_HI_STREAM = []


def _compute_stream(high):
    """bench --ab cprio_hi / cprio_def: run the step on a high-priority stream (the data-gradient chain's
    blocks dispatched ahead of the weight-gradient stream's) or on the default stream."""
    import torch

    torch.cuda.synchronize()
    if high:
        if not _HI_STREAM:
            _HI_STREAM.append(torch.cuda.Stream(priority=-1))
        torch.cuda.set_stream(_HI_STREAM[0])
    else:
        torch.cuda.set_stream(torch.cuda.default_stream())


_AB = {
    "cprio_hi": lambda: _compute_stream(True),
    "cprio_def": lambda: _compute_stream(False),
    "dks1": lambda: _set_flag("hetseq_amd.runtime.streams", "DGRAD_KSPLIT", 1),  # data-gradient K split
    "dks2": lambda: _set_flag("hetseq_amd.runtime.streams", "DGRAD_KSPLIT", 2),
    "fks_auto": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_KS", None),  # forward chains' K split
    "fks1": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_KS", 1),
    "fks2": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_KS", 2),
    "fks4": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_KS", 4),
    "fsplit_on": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_SPLIT", True),  # half-batch forward chains
    "fsplit_off": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_SPLIT", False),
    "stag0": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_STAGGER", 0),  # forward chains in phase
    "stag1": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_STAGGER", 1),  # ... second after the QKV product
    "stag2": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_STAGGER", 2),  # ... after the attention
    "stag3": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_STAGGER", 3),  # ... after the first LayerNorm
    # h3p LN forward: split-K slab count at compile time (every load of a row in flight) / runtime loop
    "lnns_on": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_fwd_ns(1),
    "lnns_off": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_fwd_ns(0),
    "attds_on": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_ATTN_DS", True),  # dQ from the stored dS
    "attds_off": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_ATTN_DS", False),  # ... or the fused dQ role
    "defer_on": lambda: setattr(__import__("hetseq_amd.parallel.ddp", fromlist=["x"]).FlatDDP, "DEFER_LAST_EARLY", True),
    "defer_off": lambda: setattr(__import__("hetseq_amd.parallel.ddp", fromlist=["x"]).FlatDDP, "DEFER_LAST_EARLY", False),
    "fsplit_bf16_on": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_SPLIT_BF16", True),  # bf16 half-batch chains
    "fsplit_bf16_off": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FWD_SPLIT_BF16", False),
    "wks2": lambda: _set_side_ks(2, 4),  # side-stream weight-gradient K split (default), small products 4
    "wks4": lambda: _set_side_ks(4, 4),  # 4 slices for every weight gradient
    "wks2s2": lambda: _set_side_ks(2, 2),
    "wks1": lambda: _set_side_ks(1, 1),  # no split-K (no reduce pass, fewer longer blocks)
    "wks1s4": lambda: _set_side_ks(1, 4),
    "lnp_on": lambda: _set_ln_partials(True),    # FFN-out split-K partials summed in the LN forward
    "lnp_off": lambda: _set_ln_partials(False),  # ... or reduced by the GEMM's own pass
    "lnb_chunk": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_bwd_lds(1),  # 3 KB LDS
    "lnb_full": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_bwd_lds(0),   # 12 KB LDS
    "fork_co": lambda: _set_flag("hetseq_amd.runtime.streams", "COALESCE", True),  # one event per fork point
    "fork_each": lambda: _set_flag("hetseq_amd.runtime.streams", "COALESCE", False),  # one per side launch
    "swf0": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_stream_wait_flags(0),
    "swf1": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_stream_wait_flags(1),
    "wcol_on": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_WGRAD_COLSUM", True),  # QKV bias grad in the wgrad
    "wcol_off": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_WGRAD_COLSUM", False),  # separate column sum
    "head_hip": lambda: _set_head_engine("hip"),  # the MLM transform's 640-row products on the split-bf16 kernel
    "head_blas": lambda: _set_head_engine("blas"),  # ... or the library (the isolated measurement's choice)
    "fresh_on": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FRESH_WGRAD", True),  # store after zero_grad
    "fresh_off": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_FRESH_WGRAD", False),  # always accumulate
    "ddec8": lambda: _set_decoder_dgrad_ks(8),  # K split of the tied decoder's data gradient (K = vocab)
    "ddec16": lambda: _set_decoder_dgrad_ks(16),
    "ddec32": lambda: _set_decoder_dgrad_ks(32),
    # K split of the half-batch FFN-out product (h3 engine; its partials go to the LN forward)
    "fo_ks2": lambda: _set_site_ks((2048, 768, 3072, False, True, 0, False), 2),
    "fo_ks4": lambda: _set_site_ks((2048, 768, 3072, False, True, 0, False), 4),
    "lnpo_on": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_LN_PARTIALS_WO", True),  # attention-output part
    "lnpo_off": lambda: _set_flag("hetseq_amd.ops.bert_ops", "_LN_PARTIALS_WO", False),
    # h3 GEMMs at three blocks per CU: all plain products / forward / data gradients / weight gradients
    "occ3_on": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_h3_occ3(7),
    "occ3_off": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_h3_occ3(0),
    "occ3_f": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_h3_occ3(1),
    "occ3_d": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_h3_occ3(2),
    "occ3_w": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_h3_occ3(4),
    "occ3_fw": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_h3_occ3(5),
    # fp32 attention engine: h3 (split-fp16, default) / native (exact fp32)
    "attn_native": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_attn_fp32_mode(0),
    "attn_h3": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_attn_fp32_mode(2),
    "adam_8k": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_adam_config(8192, 2, 1),
    "adam_64k": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_adam_config(65536, 2, 1),
    # split-K of the side-stream weight gradients (runtime/streams.py): the default 2 (4 for <= 768 x 768)
    "sideks_2": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "SIDE_KSPLIT", 2),
    "sideks_1": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "SIDE_KSPLIT", 1),
    "sideks_4": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "SIDE_KSPLIT", 4),
    "ffnbias_wgrad": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_FFN_BIAS_WGRAD", True),
    "ffnbias_dgelu": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_FFN_BIAS_WGRAD", False),
    "wcolfold_on": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_wcol_fold(1),
    "wcolfold_off": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_wcol_fold(0),
    "cfork_on": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "FWD_CHAIN_FORK", True),
    "cfork_off": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "FWD_CHAIN_FORK", False),
    "chain_on": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "FWD_CHAIN", True),
    "chain_off": lambda: setattr(__import__("hetseq_amd.runtime.streams", fromlist=["x"]), "FWD_CHAIN", False),
    "wamax_split": lambda: setattr(__import__("hetseq_amd.ops.gemm", fromlist=["x"]), "_SPLIT_WEIGHT_AMAX", True),
    "wamax_inline": lambda: setattr(__import__("hetseq_amd.ops.gemm", fromlist=["x"]), "_SPLIT_WEIGHT_AMAX", False),
    "fwdks_auto": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_FWD_KS", None),
    "fwdks_1": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_FWD_KS", 1),
    "fwdks_2": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_FWD_KS", 2),
    "poolw_side": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_POOL_WGRAD_SIDE", True),
    "poolw_inline": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_POOL_WGRAD_SIDE", False),
    "lazyzero_on": lambda: setattr(__import__("hetseq_amd.controller", fromlist=["x"]), "_LAZY_ZERO", True),
    "lazyzero_off": lambda: setattr(__import__("hetseq_amd.controller", fromlist=["x"]), "_LAZY_ZERO", False),
    # fp32 product engine of the encoder layers: h3p (pre-split block-scaled planes) / h3 (in-kernel split)
    "eng_h3p": lambda: __import__("hetseq_amd.ops.gemm", fromlist=["x"]).set_fp32_mode("h3p"),
    # staged update: the optimizer chunks on their own stream, overlapped with the next forward
    "staged_on": lambda: setattr(_CTL[0].optimizer, "staged", _CTL[0]._staged_ok()),
    "staged_off": lambda: (_CTL[0].store.params_ready(), setattr(_CTL[0].optimizer, "staged", False)),
    # K slices of the h3p forward's N = 768 products (ops/bert_ops.py _H3P_KS_WO / _H3P_KS_W2)
    "wo_ks1": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_WO", 1),
    "wo_ks2": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_WO", 2),
    "wo_ks4": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_WO", 4),
    "w2_ks1": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_W2", 1),
    "w2_ks2": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_W2", 2),
    "w2_ks4": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_W2", 4),
    "w2_ks8": lambda: setattr(__import__("hetseq_amd.ops.bert_ops", fromlist=["x"]), "_H3P_KS_W2", 8),
    # waves per 32-row block of the h3p LayerNorm forward
    "lnw8": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_h3p_waves(8),
    "lnw16": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_h3p_waves(16),
    # diagnostic ablation (results invalid): skip the split-K finishing passes / the column reductions
    "skip_none": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_skip_launches(0),
    "skip_splitk": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_skip_launches(1),
    "skip_reduce": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_skip_launches(2),
    "skip_both": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_skip_launches(3),
    "attf_auto": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_attn_h3_variant(-1, 2),
    "attf_pair": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_attn_h3_variant(1, 2),
    "attf_tile": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_attn_h3_variant(0, 2),
    "head_h3p": lambda: setattr(__import__("hetseq_amd.models.bert", fromlist=["x"]), "HEAD_H3P", True),
    "head_h3": lambda: setattr(__import__("hetseq_amd.models.bert", fromlist=["x"]), "HEAD_H3P", False),
    "lnw0": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_h3p_waves(0),
    "lnw1": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_h3p_waves(1),
    "lnbc_on": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_bwd_coop(1),
    "lnbc_off": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_bwd_coop(0),
    "lnbc_4": lambda: __import__("hetseq_amd.ops._C", fromlist=["hip"]).hip().set_ln_bwd_coop(2),
    "eng_h3": lambda: __import__("hetseq_amd.ops.gemm", fromlist=["x"]).set_fp32_mode("h3"),
    # --emulate-world: workgroups per emulated collective (RCCL channels) and the emulated bus bandwidth
    "emu_ch4": lambda: _set_emul_channels(4),
    "emu_ch8": lambda: _set_emul_channels(8),
    "emu_ch16": lambda: _set_emul_channels(16),
    "emu_ch32": lambda: _set_emul_channels(32),
    "emu_ch64": lambda: _set_emul_channels(64),
    "emu_bw250": lambda: _set_emul_busbw(250.0),
    "emu_bw400": lambda: _set_emul_busbw(400.0),
    "emu_bw600": lambda: _set_emul_busbw(600.0),
}


def _comm_identity(ctl, world, rank):
    """Per rank, before timing: the PCI bus id of the device it runs on and -- on the native engine --
    what RCCL itself reports for the communicator (ncclCommCount / ncclCommUserRank / its device) and
    the bus bandwidth of a 64 MB all-reduce.  Rank 0 checks that the job is N ranks on N DISTINCT
    devices and that RCCL saw N ranks 0..N-1 (a misconfigured launch fails here, not in the result)."""
    import torch
    import torch.distributed as dist

    from hetseq_amd.ops._C import hip

    dev = torch.cuda.current_device()
    me = {"rank": rank, "hip_device": dev, "pci_bus_id": hip().pci_bus_id(dev)}
    comm = getattr(ctl.model, "comm", None)
    if comm is not None:
        me.update(comm.identity())
        me["allreduce_64mb_busbw_gbs"] = comm.busbw(64 << 20)
    ids = [me]
    if world > 1:
        ids = [None] * world
        dist.all_gather_object(ids, me)
        buses = {i["pci_bus_id"] for i in ids}
        # (gloo runs may share a device on purpose: the one-GPU multi-rank tests; RCCL never does)
        if rank == 0 and len(buses) != world and dist.get_backend() == "nccl":
            raise RuntimeError("bench.py: %d ranks on %d distinct devices: %s" % (world, len(buses), ids))
        if rank == 0:
            if comm is not None and (any(i.get("rccl_count") != world for i in ids)
                                     or sorted(i.get("rccl_rank") for i in ids) != list(range(world))):
                raise RuntimeError("bench.py: RCCL does not see %d ranks 0..%d: %s" % (world, world - 1, ids))
    return ids


def _host_phases(ctl):
    """Wrap the phases of train_step with host timers (diagnostic, --host-phases): where the host
    spends -- or waits out -- its time per step."""
    acc = {}

    def timed(obj, name, label):
        fn = getattr(obj, name)

        def wrapper(*a, **k):
            t = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                d = time.perf_counter() - t
                s_, m_ = acc.get(label, (0.0, 0.0))
                acc[label] = (s_ + d, max(m_, d))
        setattr(obj, name, wrapper)

    timed(ctl.model, "forward", "forward")
    timed(ctl.optimizer, "backward", "backward")
    timed(ctl.optimizer, "clip_grad_norm", "grad_norm")
    timed(ctl.optimizer, "step", "optimizer_step")
    timed(ctl, "zero_grad", "zero_grad")
    timed(ctl, "_prepare_sample", "prepare_sample")
    timed(ctl, "_set_seed", "set_seed")
    return acc


_CTL = [None]  # the controller of an --ab run (variants that switch its state)


def _ab_run(b, ctl, gen):
    import torch

    _CTL[0] = ctl
    names = b.ab.split(",")
    times = {n: [] for n in names}
    for r in range(b.ab_rounds):
        for n in (names if r % 2 == 0 else names[::-1]):  # alternate the order too
            for part in n.split("+"):  # "a+b": both settings
                _AB[part]()
            ctl.train_step(next(gen))  # one untimed step after a switch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(b.steps):
                ctl.train_step(next(gen))
            torch.cuda.synchronize()
            times[n].append((time.perf_counter() - t0) / b.steps * 1000)
    out = {n: {"median_ms": round(sorted(v)[len(v) // 2], 3), "all": [round(x, 3) for x in v]} for n, v in times.items()}
    sys.stdout.write(json.dumps({"ab": out, "steps_per_segment": b.steps, "rounds": b.ab_rounds}) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
