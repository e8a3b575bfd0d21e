"""Data-parallel engine on the GPU path (fused kernels + FlatDDP) with 2 ranks.

The box has one GPU, and RCCL refuses two ranks on one device, so both ranks
share GPU 0 over the gloo backend (CUDA tensors).  This exercises the real
GPU-side flow -- fused backward writing gradients straight into the flat
buffer, readiness notifications, in-order async bucket all-reduces, the
stats all-reduce -- and checks parameter consistency every update.
"""
import os
import sys

import pytest

from tests.test_distributed_cpu import ROOT, _free_port

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def test_two_ranks_fused_bert_on_one_gpu(tmp_path):
    import subprocess

    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab

    d = tmp_path / "bert"
    write_bert_shards(str(d), num_shards=2, per_shard=64, seq_len=64, max_pred=8, vocab_size=1000, split="train")
    write_bert_shards(str(d), num_shards=1, per_shard=8, seq_len=64, max_pred=8, vocab_size=1000, split="test")
    write_vocab(str(tmp_path / "vocab.txt"), 1000)
    cfg = write_bert_config(str(tmp_path / "cfg.json"), vocab_size=1000, hidden_size=256, num_hidden_layers=2,
                            num_attention_heads=4, intermediate_size=1024)
    init = "tcp://127.0.0.1:%d" % _free_port()
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    cmds = [[sys.executable, os.path.join(ROOT, "train.py"), "--task", "bert", "--data", str(d), "--dict",
             str(tmp_path / "vocab.txt"), "--config_file", cfg, "--max-sentences", "8", "--valid-subset", "test",
             "--max-update", "6", "--distributed-backend", "gloo", "--save-dir", str(tmp_path / "ck"),
             "--distributed-init-method", init, "--distributed-world-size", "2", "--distributed-rank", str(r),
             "--distributed-gpus", "1", "--device-id", "0", "--check-consistency", "1", "--fast-stat-sync",
             "--lr", "1e-3", "--bucket-cap-mb", "1"] for r in range(2)]
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env) for c in cmds]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=400)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    assert "(epoch 1 @ 6 updates)" in outs[0]


def test_bert_resume_mid_epoch_matches_uninterrupted(tmp_path):
    """train.py on the fused GPU path: 3 updates, stop, resume from checkpoint_last.pt to 6 updates
    == 6 updates in one run (same parameters, optimizer state and iterator position; deterministic
    kernels, per-update dropout seeds)."""
    import subprocess

    import torch

    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab

    d = tmp_path / "bert"
    write_bert_shards(str(d), num_shards=2, per_shard=64, seq_len=64, max_pred=8, vocab_size=1000, split="train")
    write_bert_shards(str(d), num_shards=1, per_shard=8, seq_len=64, max_pred=8, vocab_size=1000, split="test")
    write_vocab(str(tmp_path / "vocab.txt"), 1000)
    cfg = write_bert_config(str(tmp_path / "cfg.json"), vocab_size=1000, hidden_size=256, num_hidden_layers=2,
                            num_attention_heads=4, intermediate_size=1024)
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["HETSEQ_GEMM"] = "hip"  # no timing-based engine choice between the runs

    def run(save_dir, max_update):
        cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--task", "bert", "--data", str(d), "--dict",
               str(tmp_path / "vocab.txt"), "--config_file", cfg, "--max-sentences", "8", "--max-update",
               str(max_update), "--save-dir", str(save_dir), "--distributed-world-size", "1", "--fast-stat-sync",
               "--valid-subset", "test",
               "--lr", "1e-3", "--warmup-updates", "2", "--log-format", "simple", "--log-interval", "1"]
        p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, timeout=300)
        assert p.returncode == 0, p.stdout[-3000:]
        return p.stdout

    run(tmp_path / "a", 6)
    run(tmp_path / "b", 3)
    out = run(tmp_path / "b", 6)
    assert "loaded checkpoint" in out, out[-2000:]
    sa = torch.load(str(tmp_path / "a" / "checkpoint_last.pt"), map_location="cpu", weights_only=False)
    sb = torch.load(str(tmp_path / "b" / "checkpoint_last.pt"), map_location="cpu", weights_only=False)
    assert sa["optimizer_history"][-1]["num_updates"] == sb["optimizer_history"][-1]["num_updates"] == 6
    for k, v in sa["model"].items():
        assert torch.equal(v, sb["model"][k]), k
    ea, eb = sa["last_optimizer_state"]["state"], sb["last_optimizer_state"]["state"]
    for i in ea:
        assert torch.equal(ea[i]["exp_avg"], eb[i]["exp_avg"]) and torch.equal(ea[i]["exp_avg_sq"], eb[i]["exp_avg_sq"])


def test_bench_self_launches_two_ranks(tmp_path):
    """``python bench.py --gpus 2`` with no launcher: the parent starts two rank processes (never
    touching the GPU itself), they time BERT-base data-parallel steps, rank 0 reports n_gpus 2 /
    dp2.  Two ranks share the box's one GPU over gloo (RCCL refuses two ranks on one device)."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--steps", "5", "--warmup", "2"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 64
    assert out["config"]["comm"] == "c10d-gloo" and out["steps"] == 5
    assert out["value"] > 0


def test_bench_hetero_device_map_from_rank_processes(tmp_path):
    """``bench.py --hetero 1,2 --dist-backend gloo``: two launch groups (1 + 2 ranks, tcp:// rendezvous)
    of real rank processes.  gloo keeps all three on GPU 0 (``ran_on``), but each rank computes and
    reports the device the nccl path would use -- group offset + local index (reference
    train.py:189-193, Q24 fix): ranks 0 / 1 / 2 -> devices 0 / 1 / 2, local ranks 0 / 0 / 1."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--hetero", "1,2", "--dist-backend", "gloo",
                        "--steps", "1", "--warmup", "1", "--layers", "1"], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][-1]
    assert out["n_gpus"] == 3 and "hetero 1+2" in out["config"]["parallelism"]
    dm = out["device_map"]
    assert [d["rank"] for d in dm] == [0, 1, 2]
    assert [d["group"] for d in dm] == [0, 1, 1]
    assert [d["local_rank"] for d in dm] == [0, 0, 1]
    assert [d["device_id"] for d in dm] == [0, 1, 2]
    assert all(d["ran_on"] == 0 for d in dm)


def _tied_worker(rank, port, q, sparse):
    try:
        import torch
        import torch.distributed as dist

        from hetseq_amd.parallel.ddp import FlatDDP
        from hetseq_amd.runtime.flat import FlatParamStore
        from tests.test_bert_gpu import _batch, _tiny

        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, world_size=2, rank=rank)
        cuda = torch.device("cuda", 0)
        torch.cuda.set_device(cuda)
        model, cfg = _tiny(cuda)
        model.eval()
        model.max_predictions_per_seq = 10
        store = FlatParamStore(model)
        model.attach_store(store, torch.float32)
        net = FlatDDP(model, store, bucket_cap_mb=0.25, comm_engine="c10d",
                      sparse_embedding=model.sparse_embedding() if sparse else None)
        assert (net.tables is not None) == sparse
        ids, tt, mask, labels, nsp = _batch(cuda, 4, 64, cfg.vocab_size)
        ids = (ids + 37 * rank) % cfg.vocab_size  # different tokens per rank, some shared
        store.zero_grad()  # opens the fresh-gradient window (store-mode weight gradients)
        for micro in range(2):  # update_freq 2: a no_sync micro-batch first (dense local tables)
            with (net.no_sync() if micro == 0 else torch.enable_grad()):
                net(ids, tt, mask, labels, nsp).backward()
        torch.cuda.synchronize()
        q.put((rank, store.grad.cpu().numpy().copy(), [w for w, _, late, _ in net.comm_log if late]))
        dist.destroy_process_group()
    except BaseException as e:
        q.put((rank, None, repr(e)))
        raise


def test_tied_tables_sparse_exchange_two_ranks_fused_bert():
    """Fused BERT backward, 2 ranks sharing the GPU over gloo (c10d engine): the sparse table
    exchange (early dense bucket + row gather + sorted-run scatter, parallel/tied.py) gives the
    dense-bucket engine's gradient, after a no_sync micro-batch too, with identical replicas."""
    import multiprocessing as mp

    import torch

    res = {}
    for sparse in (True, False):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_tied_worker, args=(r, port, q, sparse)) for r in range(2)]
        for p in procs:
            p.start()
        out = {}
        for _ in range(2):
            r, g, tail = q.get(timeout=300)
            assert g is not None, "rank %d: %s" % (r, tail)
            out[r] = (torch.from_numpy(g), tail)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        res[sparse] = out
    g_sp, g_dn = res[True][0][0], res[False][0][0]
    assert torch.equal(g_sp, res[True][1][0])
    assert torch.equal(g_dn, res[False][1][0])
    assert torch.allclose(g_sp, g_dn, rtol=1e-5, atol=1e-6), (g_sp - g_dn).abs().max().item()
    assert res[True][0][1][0] == "rows", res[True][0][1]


def test_bench_two_ranks_gloo_bf16_hip_graph(tmp_path):
    """``bench.py --gpus 2 --dist-backend gloo --dtype bf16 --hip-graph``: data-parallel over c10d
    runs the split-graph path (forward+backward graph, eager gradient exchange, update graph)."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--dtype", "bf16", "--hip-graph", "--steps", "5", "--warmup", "4"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")][0]
    assert out["n_gpus"] == 2 and out["config"]["hip_graph"] is True and out["dtype"] == "bf16"
    assert out["value"] > 0
