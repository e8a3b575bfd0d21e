"""Native RCCL engine (csrc/comm/comm.cpp) on one MI355X: a 1-rank communicator.

Multi-rank RCCL needs one GPU per rank (RCCL refuses two ranks on one device), so
the multi-rank semantics are covered by the CPU/gloo suites through the same
FlatDDP code path; here the engine's own mechanics run for real: unique-id
rendezvous through the process-group store, in-stream collectives, event-gated
bucket all-reduces on the greatest-priority comm stream with the consumer join,
the watchdog abort (injected stall), and FlatDDP driving it through a backward
that uses the weight-gradient side stream.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def group(cuda_module):
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), world_size=1, rank=0)
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def cuda_module():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from hetseq_amd.parallel import comm

    if comm.module() is None:
        pytest.fail("hetseq_amd._comm is not built")  # loud: the native engine must be present on a GPU box
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def test_collectives_single_rank(group):
    from hetseq_amd.parallel.comm import NativeComm

    c = NativeComm(group, timeout_s=60)
    try:
        x = torch.arange(1000, dtype=torch.float32, device="cuda")
        assert torch.equal(c.all_reduce(x.clone()), x)
        s = torch.tensor([1.5, 2.5, 3.0, 4.0, 5.0, 0.0], dtype=torch.float64, device="cuda")
        assert torch.equal(c.all_reduce(s.clone()), s)
        assert torch.equal(c.all_reduce(x.clone(), op="max"), x)
        b = torch.randn(257, device="cuda").bfloat16()
        assert torch.equal(c.broadcast(b.clone()), b)
        out = torch.empty(300, dtype=torch.int64, device="cuda")
        src = torch.arange(300, device="cuda")
        assert torch.equal(c.all_gather(out, src), src)
        c.check()
    finally:
        c.close()


def test_identity_reports_rccl_view(group):
    """What bench.py records per rank: RCCL's own count / rank / device for the communicator and
    the device's PCI bus id (here: 1 rank), and a positive 64 MB all-reduce bandwidth."""
    from hetseq_amd.ops._C import hip
    from hetseq_amd.parallel.comm import NativeComm

    c = NativeComm(group, timeout_s=60)
    try:
        ident = c.identity()
        assert ident["rccl_count"] == 1 and ident["rccl_rank"] == 0
        assert ident["rccl_device"] == torch.cuda.current_device()
        assert ident["pci_bus_id"] == hip().pci_bus_id(torch.cuda.current_device()) and ident["pci_bus_id"]
        assert c.busbw(8 << 20, iters=2) > 0
    finally:
        c.close()


def test_async_bucket_ordering(group):
    """The comm stream must wait for the producer stream (a long kernel writes the bucket) and
    the consumer must wait for the comm stream: the result equals the producer's output."""
    from hetseq_amd.parallel.comm import NativeComm

    c = NativeComm(group, timeout_s=60)
    try:
        n = 1 << 22
        g = torch.zeros(n, device="cuda")
        a = torch.randn(2048, 2048, device="cuda")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(8):  # keep the producer busy so an unordered collective would read zeros
                a = torch.tanh(a @ a * 1e-3)
            g.fill_(3.0)
        c.all_reduce_async(g, producers=(torch.cuda.current_stream(), side))
        c.wait()
        got = g.sum().item()
        assert got == 3.0 * n
        torch.cuda.synchronize()
        assert c.outstanding() <= 1  # the watchdog retires completed operations
    finally:
        c.close()


def test_watchdog_aborts_stuck_collective(group):
    from hetseq_amd.parallel.comm import NativeComm

    c = NativeComm(group, timeout_s=0.3)
    c.inject_stall(1)
    c.all_reduce(torch.ones(16, device="cuda"))
    deadline = time.time() + 10
    while not c.aborted and time.time() < deadline:
        time.sleep(0.05)
    assert c.aborted
    with pytest.raises(RuntimeError, match="aborted"):
        c.check()
    with pytest.raises(RuntimeError, match="aborted"):
        c.all_reduce(torch.ones(16, device="cuda"))
    c.close()


def test_flatddp_native_engine_matches_local(group):
    """FlatDDP over the native engine (1 rank: the all-reduce is an identity) reproduces the
    local gradients bit for bit, through the fused BERT path whose weight gradients run on the
    side stream (bucket all-reduces gated on both producer streams)."""
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    grads = []
    old = streams.enabled()
    streams.set_enabled(True)
    try:
        for engine in ("local", "native"):
            model, cfg = _tiny(cuda)
            model.eval()
            model.max_predictions_per_seq = 10
            store = FlatParamStore(model)
            model.attach_store(store, torch.float32)
            net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="native", timeout_s=60) \
                if engine == "native" else model
            if engine == "native":
                assert net.comm is not None and len(net.buckets) > 3
            batch = _batch(cuda, 4, 64, cfg.vocab_size)
            store.grad.zero_()
            net(*batch).backward()
            torch.cuda.synchronize()
            grads.append(store.grad.clone())
            if engine == "native":
                net.comm.check()
                net.comm.close()
    finally:
        streams.set_enabled(old)
    assert torch.equal(grads[0], grads[1])


def _snapshot_run(group, gate_side_stream):
    """Fused BERT backward through FlatDDP on the native engine in snapshot mode, with the
    weight-gradient side stream delayed so an ungated bucket copy would see unfinished grads.
    Returns (snapshot, final gradient, bucket ranges)."""
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    model, cfg = _tiny(cuda)
    model.eval()
    model.max_predictions_per_seq = 10
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="native", timeout_s=60)
    snap = torch.full_like(store.grad, float("nan"))
    net.comm.set_snapshot(snap, store.grad)
    orig_fork, orig_active = streams.fork, streams.active

    def slow_fork(device, *tensors):  # every side-stream task starts ~1 ms late
        s = orig_fork(device, *tensors)
        with torch.cuda.stream(s):
            torch.cuda._sleep(2_000_000)
        return s

    streams.fork = slow_fork
    if not gate_side_stream:  # remove the side-stream producer event from the bucket launches
        streams.active = lambda device: None
    try:
        batch = _batch(cuda, 4, 64, cfg.vocab_size)
        store.grad.zero_()
        net(*batch).backward()
        torch.cuda.synchronize()
    finally:
        streams.fork, streams.active = orig_fork, orig_active
        net.comm.set_snapshot(None, None)
        net.comm.check()
        net.comm.close()
    return snap, store.grad.clone(), net.ranges


def test_bucket_snapshots_equal_final_gradients(group):
    """Every bucket, copied on the comm stream exactly when its all-reduce would read it, already
    holds its final gradient: the producer events on BOTH streams (compute and weight-gradient)
    gate the launch.  Control: without the side-stream event the same run snapshots unfinished
    buckets, so this test would catch a missing producer event."""
    from hetseq_amd.runtime import streams

    old = streams.enabled()
    streams.set_enabled(True)
    try:
        snap, grad, ranges = _snapshot_run(group, True)
        for lo, hi in ranges:
            assert torch.equal(snap[lo:hi], grad[lo:hi]), (lo, hi)
        snap_bad, grad_bad, ranges = _snapshot_run(group, False)
        assert any(not torch.equal(snap_bad[lo:hi], grad_bad[lo:hi]) for lo, hi in ranges)
    finally:
        streams.set_enabled(old)


def test_tied_tables_early_bucket_and_sparse_rows(group):
    """Tied word-embedding tail (parallel/tied.py) on the fused BERT path, native engine in
    snapshot mode: the tables' early bucket is read (snapshot copy on the comm stream, where the
    all-reduce would read it) after the tied decoder's weight GEMM and BEFORE any embedding row is
    added -- so the position / token-type tables are still zero there and every word row no token
    touched already holds its final value; the bytes issued after the last backward kernel are the
    row gather (B*S*H*4) plus the embedding LayerNorm's 2*H*4; and the gradient equals the
    engine-free fused backward's."""
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    B, S = 4, 64
    old = streams.enabled()
    streams.set_enabled(True)
    try:
        grads = []
        for use_ddp in (False, True):
            model, cfg = _tiny(cuda)
            model.eval()
            model.max_predictions_per_seq = 10
            store = FlatParamStore(model)
            model.attach_store(store, torch.float32)
            batch = _batch(cuda, B, S, cfg.vocab_size)
            store.zero_grad()  # store-mode weight gradients + the sparse exchange
            if not use_ddp:
                model(*batch).backward()
                torch.cuda.synchronize()
                grads.append(store.grad.clone())
                continue
            net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="native", timeout_s=60,
                          sparse_embedding=model.sparse_embedding())
            assert net.tables is not None
            snap = torch.full_like(store.grad, float("nan"))
            net.comm.set_snapshot(snap, store.grad)
            try:
                net(*batch).backward()
                torch.cuda.synchronize()
            finally:
                net.comm.set_snapshot(None, None)
                net.comm.check()
                net.comm.close()
            grads.append(store.grad.clone())
            t = net.tables
            H = cfg.hidden_size
            V = cfg.vocab_size
            region_snap = snap[t.lo:t.hi].view(t.K, H)
            region = store.grad[t.lo:t.hi].view(t.K, H)
            assert torch.all(region_snap[V:] == 0)  # position + type rows: no embedding row added yet
            touched = torch.zeros(V, dtype=torch.bool, device=cuda)
            touched[batch[0].reshape(-1)] = True
            assert torch.equal(region_snap[:V][~touched], region[:V][~touched])
            assert not torch.equal(region_snap[:V][touched], region[:V][touched])
            names = [w for w, *_ in net.comm_log]
            assert names[:2] == ["keys", "allreduce_tables"], names
            tail = [(w, b) for w, b, late, _ in net.comm_log if late]
            assert tail[0] == ("rows", B * S * H * 4), tail
            # bytes RECEIVED after the last backward kernel: none at one rank (a 1-rank ring moves nothing)
            assert net.tail_bytes() == 0, tail
    finally:
        streams.set_enabled(old)
    ref, got = grads
    assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6), (got - ref).abs().max().item()


def test_engine_stream_roles_are_distinct_and_fit_hw_queues(group):
    """The data-parallel step runs on exactly four streams -- compute, weight-gradient side
    stream, the native engine's greatest-priority comm stream and the loader's copy stream (one
    per device for the whole job, not one per epoch iterator) -- all distinct and no more than
    GPU_MAX_HW_QUEUES, so each gets its own hardware queue (profiles/r3_stream_queues.md shows
    the placement and overlap from a kernel trace)."""
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    old = streams.enabled()
    streams.set_enabled(True)
    try:
        model, cfg = _tiny(cuda)
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="native", timeout_s=60,
                      sparse_embedding=model.sparse_embedding())
        copy = streams.copy_stream(cuda)
        assert streams.copy_stream(cuda) is copy  # a second epoch iterator reuses it
        for _ in range(2):
            store.grad.zero_()
            net(*_batch(cuda, 4, 64, cfg.vocab_size)).backward()
        torch.cuda.synchronize()
        roles = streams.engine_streams(cuda)
        roles["comm"] = net.comm.stream_handle
        net.comm.check()
        net.comm.close()
    finally:
        streams.set_enabled(old)
    assert set(roles) == {"compute", "wgrad", "copy", "comm"}, roles
    assert len(set(roles.values())) == 4, roles
    assert len(roles) <= int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))


def test_graph_captured_dp_step_matches_eager(group):
    """HIP-graph capture of a data-parallel backward on the native engine (1-rank communicator):
    the bucket all-reduces, the tables' early bucket, the key / row gathers and the stream joins
    are captured; replays give the eager step's gradient, and the watchdog registered nothing
    during capture (its events would never complete outside the graph)."""
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import streams
    from hetseq_amd.runtime.flat import FlatParamStore
    from hetseq_amd.runtime.graphs import GraphedStep
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    old = streams.enabled()
    streams.set_enabled(True)
    try:
        model, cfg = _tiny(cuda)
        model.eval()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="native", timeout_s=60,
                      sparse_embedding=model.sparse_embedding())
        batch = list(_batch(cuda, 4, 64, cfg.vocab_size))
        for _ in range(2):  # eager warm-up (capacity agreement, buffers, GEMM choices)
            store.grad.zero_()
            net(*batch).backward()
        torch.cuda.synchronize()
        eager = store.grad.clone()

        def body(inputs):
            store.grad.zero_()
            net(*inputs).backward()
            return (store.grad,)

        step = GraphedStep(body, capture_error_mode="thread_local")
        outs = [step.run(batch)[0] for _ in range(3)]
        net.comm.watch()
        torch.cuda.synchronize()
        net.comm.check()
        assert step.graph is not None
        names = [w for w, *_ in net.comm_log]  # the captured step's collectives
        assert names[:2] == ["keys", "allreduce_tables"] and "rows" in names, names
        net.comm.close()
    finally:
        streams.set_enabled(old)
    for g in outs:
        assert torch.equal(g, eager), (g - eager).abs().max().item()


def test_emulated_collectives_timing_and_identity(group):
    """bench.py --emulate-world: on the 1-rank engine every bucket all-reduce becomes the stand-in
    kernel -- the bucket is left exactly as it was (a 1-rank all-reduce is the identity), the comm
    stream is busy for at least latency + received bytes / bus bandwidth of a W-rank ring, and the
    consumer join still orders after it; world 1 restores the real collective."""
    from hetseq_amd.parallel.comm import NativeComm

    c = NativeComm(group, timeout_s=60)
    try:
        n = 8 << 20  # 32 MB bucket
        g = torch.randn(n, device="cuda")
        ref = g.clone()
        W, bw, lat = 8, 200.0, 20.0
        c.set_emulation(W, channels=16, busbw_gbs=bw, latency_us=lat)
        comm_stream = torch.cuda.ExternalStream(c.stream_handle)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record(comm_stream)
        c.all_reduce_async(g)
        e.record(comm_stream)
        c.wait()
        torch.cuda.synchronize()
        want_ms = (lat * 1e3 + 2 * (W - 1) * n * 4 / W / bw) / 1e6  # bytes / (GB/s) = ns
        got_ms = s.elapsed_time(e)
        assert got_ms >= 0.95 * want_ms, (got_ms, want_ms)
        assert got_ms < want_ms + 5.0, (got_ms, want_ms)
        assert torch.equal(g, ref)
        # the all-gather: the real 1-rank gather, then the other W-1 ranks' rows over the links
        rows = torch.randn(4096, 768, device="cuda")
        out = torch.empty_like(rows)
        s.record(comm_stream)
        c.all_gather_async(out, rows)
        e.record(comm_stream)
        c.wait()
        torch.cuda.synchronize()
        assert torch.equal(out, rows)
        assert s.elapsed_time(e) >= 0.95 * (lat * 1e3 + (W - 1) * rows.numel() * 4 / bw) / 1e6
        c.set_emulation(1)
        x = torch.arange(64, dtype=torch.float32, device="cuda")
        c.all_reduce_async(x)
        c.wait()
        torch.cuda.synchronize()
        assert torch.equal(x, torch.arange(64, dtype=torch.float32, device="cuda"))
        c.check()
    finally:
        c.close()


def test_bench_emulate_world_reports(tmp_path):
    """bench.py --emulate-world 8 runs the DP engine on one GPU with emulated collectives and says so."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1", "--layers", "2",
                        "--emulate-world", "8", "--comm-channels", "8"], capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["comm_emulated"] == 8 and out["n_gpus"] == 1
    assert out["emulation"]["channels"] == 8
    assert "emulating dp8" in out["config"]["parallelism"]
    dc = out["dp_collectives"]
    assert dc["n"] > 0 and dc["received_mb"] > dc["payload_mb"]  # 2(W-1)/W > 1 at W = 8


@pytest.mark.parametrize("delay", [0, 4_000_000])
def test_sharded_early_buckets_snapshot_and_update(group, delay):
    """Sharded update on the native engine (1 rank) with the layer program's per-group readiness
    events: every reduce-scatter region -- the early layer's four groups included, with the side
    stream held back -- reads the final gradient (snapshot mode), and an update step through the
    shard plan equals the unsharded update."""
    from argparse import Namespace

    from hetseq_amd.ops import bert_ops
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.optim.optimizers import _Adam
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import rng
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    G.set_fp32_mode("h3p")
    out = {}
    for shard in (False, True):
        model, cfg = _tiny(cuda)
        model.train()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        net = FlatDDP(model, store, comm_engine="native", timeout_s=60, shard_optimizer=shard)
        opt = _Adam(Namespace(lr=[1e-3], adam_betas="(0.9,0.999)", adam_eps=1e-8, weight_decay=0.01),
                    list(model.parameters()), store)
        if shard:
            assert store.shard is not None and len(net.early) == 4
            snap = torch.full_like(store.grad, float("nan"))
            net.comm.set_snapshot(snap, store.grad)
        bert_ops._PROG_SIDE_DELAY = delay
        try:
            opt.zero_grad()
            rng.set_seed(7)
            net(*_batch(cuda, 16, 64, cfg.vocab_size)).backward()
        finally:
            bert_ops._PROG_SIDE_DELAY = 0
        torch.cuda.synchronize()
        if shard:
            net.comm.set_snapshot(None, None)
            for lo, hi in net.ranges:
                assert torch.equal(snap[lo:hi], store.grad[lo:hi]), (lo, hi)
            assert any(p.rows == 16 * 64 for blk in model.bert.encoder.layer for p in blk.__dict__.get("_hs_progs", {}).values())
        opt.clip_grad_norm(1.0)
        opt.staged = shard  # the sharded step staged: Adam and the chunk all-gathers on the comm stream
        opt.step()
        cs = store.checksum()  # straight after the staged step: must wait for the pending gathers
        opt.state_dict()
        torch.cuda.synchronize()
        out[shard] = store.param.clone()
        assert float(cs) == float(store.param.double().sum())
        if shard:  # the engine's self-test of the in-place collectives the sharded update uses
            from hetseq_amd.parallel import comm as native_comm

            assert native_comm.shard_self_test(net.comm, group) == (True, None)
        net.comm.check()
        net.comm.close()
    assert torch.allclose(out[True], out[False], rtol=1e-6, atol=1e-7), (out[True] - out[False]).abs().max().item()


@pytest.mark.parametrize("defer", [True, False])
def test_sharded_tables_deferred_early_group(group, defer):
    """Sharded update + sparse table exchange on the native engine (1 rank, snapshot mode): with
    DEFER_LAST_EARLY the early layer's last gradient group is reduce-scattered after the embedding
    rows' all-gather (parallel/ddp.py launch_deferred_early), otherwise before it; either way every
    reduce-scatter region reads its final gradient and the gradient equals the other order's."""
    from hetseq_amd.ops import gemm as G
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime import rng
    from hetseq_amd.runtime.flat import FlatParamStore
    from tests.test_bert_gpu import _batch, _tiny

    cuda = torch.device("cuda", 0)
    G.set_fp32_mode("h3p")
    model, cfg = _tiny(cuda)
    model.train()
    model.max_predictions_per_seq = 10
    store = FlatParamStore(model)
    model.attach_store(store, torch.float32)
    net = FlatDDP(model, store, comm_engine="native", timeout_s=60, shard_optimizer=True,
                  sparse_embedding=model.sparse_embedding())
    old = FlatDDP.DEFER_LAST_EARLY
    FlatDDP.DEFER_LAST_EARLY = defer
    try:
        assert net.tables is not None and store.shard is not None and len(net.early) == 4
        snap = torch.full_like(store.grad, float("nan"))
        net.comm.set_snapshot(snap, store.grad)
        store.zero_grad()
        rng.set_seed(7)
        net(*_batch(cuda, 16, 64, cfg.vocab_size)).backward()
        torch.cuda.synchronize()
        net.comm.set_snapshot(None, None)
        names = [w for w, *_ in net.comm_log]
        last = "reducescatter_group%d" % net.early[-1]
        assert last in names and "rows" in names, names
        assert (names.index(last) > names.index("rows")) == defer, names
        for lo, hi in net.ranges:
            if hi <= net.tables.lo or lo >= net.tables.hi:  # (the tables: reduced before the rows are added)
                assert torch.equal(snap[lo:hi], store.grad[lo:hi]), (lo, hi)
        assert torch.isfinite(store.grad).all()
    finally:
        FlatDDP.DEFER_LAST_EARLY = old
        net.comm.check()
        net.comm.close()
