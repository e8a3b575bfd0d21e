"""Multi-process data parallelism on CPU/gloo through the real CLI.

Covers the reference's launch modes: separate launches per
"node" joined by file:// or tcp:// rendezvous with uneven --distributed-gpus
(the heterogeneous split), spawn mode, padded shards (dummy batches keep
ranks in lockstep), and cross-rank parameter consistency (--check-consistency
all-reduces a parameter checksum every update and fails on divergence).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    from hetseq_amd.data.synthetic import write_mnist

    d = tmp_path_factory.mktemp("mnist")
    write_mnist(str(d), n_train=200, n_test=40)  # 200/16 = 13 batches: uneven across 2 and 3 ranks
    return str(d)


def _cmd(data, save, extra):
    return [sys.executable, os.path.join(ROOT, "train.py"), "--task", "mnist", "--optimizer", "adadelta", "--lr", "1.0",
            "--data", data, "--max-sentences", "16", "--valid-subset", "test", "--max-epoch", "2", "--cpu",
            "--distributed-backend", "gloo", "--save-dir", save, "--check-consistency", "1", "--clip-norm", "0",
            "--log-format", "simple", "--log-interval", "1"] + extra


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    return env


def _run_all(cmds, timeout=300):
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=_env())
             for c in cmds]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    return [o for _, o in outs]


def _losses(out):
    import re

    return [float(m) for m in re.findall(r"loss=([0-9.]+)", out)]


def test_two_launches_file_init_fast_stat(mnist_dir, tmp_path):
    init = "file://" + str(tmp_path / "rdzv")
    save = str(tmp_path / "ckpt")
    cmds = [_cmd(mnist_dir, save, ["--distributed-init-method", init, "--distributed-world-size", "2",
                                   "--distributed-rank", str(r), "--distributed-gpus", "1", "--fast-stat-sync"])
            for r in range(2)]
    out0, out1 = _run_all(cmds)
    l0 = _losses(out0)
    assert len(l0) >= 10 and l0[-1] < l0[0]
    assert os.path.exists(os.path.join(save, "checkpoint_last.pt"))
    # with --fast-stat-sync both ranks log the same global loss (rank 1 output is suppressed)
    assert "loss=" not in out1


def test_heterogeneous_tcp_split_1_plus_2(mnist_dir, tmp_path):
    """Three ranks from two launches: node A contributes 1 worker, node B 2 (spawned)."""
    init = "tcp://127.0.0.1:%d" % _free_port()
    save = str(tmp_path / "ckpt")
    a = _cmd(mnist_dir, save, ["--distributed-init-method", init, "--distributed-world-size", "3",
                               "--distributed-rank", "0", "--distributed-gpus", "1"])
    b = _cmd(mnist_dir, save, ["--distributed-init-method", init, "--distributed-world-size", "3",
                               "--distributed-rank", "1", "--distributed-gpus", "2"])
    out_a, _ = _run_all([a, b])
    # 13 batches over 3 ranks -> 5 updates per epoch (last one padded with dummy batches)
    assert "num_updates=5," in out_a and "num_updates=10," in out_a


def test_slow_stat_path_and_update_freq(mnist_dir, tmp_path):
    init = "file://" + str(tmp_path / "rdzv")
    cmds = [_cmd(mnist_dir, str(tmp_path / "c"), ["--distributed-init-method", init, "--distributed-world-size", "2",
                                                  "--distributed-rank", str(r), "--distributed-gpus", "1",
                                                  "--update-freq", "2", "--max-epoch", "1"])
            for r in range(2)]
    out0, _ = _run_all(cmds)
    assert "num_updates=4," in out0  # ceil(7 / 2) updates for 7 batches per rank


def test_bert_tiny_two_ranks(tmp_path):
    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab

    d = tmp_path / "bert"
    write_bert_shards(str(d), num_shards=2, per_shard=24, seq_len=32, max_pred=5, vocab_size=300, split="train")
    write_bert_shards(str(d), num_shards=1, per_shard=8, seq_len=32, max_pred=5, vocab_size=300, split="test")
    write_vocab(str(tmp_path / "vocab.txt"), 300)
    cfg = write_bert_config(str(tmp_path / "cfg.json"), vocab_size=300, hidden_size=64, num_hidden_layers=2,
                            num_attention_heads=2, intermediate_size=128)
    init = "file://" + str(tmp_path / "rdzv")
    cmds = [[sys.executable, os.path.join(ROOT, "train.py"), "--task", "bert", "--data", str(d), "--dict",
             str(tmp_path / "vocab.txt"), "--config_file", cfg, "--max-sentences", "4", "--valid-subset", "test",
             "--max-update", "5", "--cpu", "--distributed-backend", "gloo", "--save-dir", str(tmp_path / "ck"),
             "--distributed-init-method", init, "--distributed-world-size", "2", "--distributed-rank", str(r),
             "--distributed-gpus", "1", "--check-consistency", "1", "--fast-stat-sync", "--lr", "1e-3",
             "--bucket-cap-mb", "1"] for r in range(2)]
    out0, _ = _run_all(cmds)
    assert "num_updates=4," in out0 and "(epoch 1 @ 5 updates)" in out0


def test_bert_tiny_eight_ranks_hetero_3_plus_5(tmp_path):
    """The driver's 8-rank data-parallel shape rehearsed on CPU/gloo: BERT (tiny) through the
    flat-store DP engine with several buckets, two heterogeneous launches (3 + 5 spawned
    processes, tcp:// rendezvous), update-freq 2 (no_sync on the first micro-batch), and a
    parameter-checksum consistency check after every update."""
    from hetseq_amd.data.synthetic import write_bert_config, write_bert_shards, write_vocab

    d = tmp_path / "bert"
    write_bert_shards(str(d), num_shards=2, per_shard=80, seq_len=32, max_pred=5, vocab_size=300, split="train")
    write_bert_shards(str(d), num_shards=1, per_shard=8, seq_len=32, max_pred=5, vocab_size=300, split="test")
    write_vocab(str(tmp_path / "vocab.txt"), 300)
    cfg = write_bert_config(str(tmp_path / "cfg.json"), vocab_size=300, hidden_size=64, num_hidden_layers=2,
                            num_attention_heads=2, intermediate_size=128)
    init = "tcp://127.0.0.1:%d" % _free_port()
    base = [sys.executable, os.path.join(ROOT, "train.py"), "--task", "bert", "--data", str(d), "--dict",
            str(tmp_path / "vocab.txt"), "--config_file", cfg, "--max-sentences", "4", "--valid-subset", "test",
            "--max-update", "3", "--cpu", "--distributed-backend", "gloo", "--save-dir", str(tmp_path / "ck"),
            "--distributed-init-method", init, "--distributed-world-size", "8", "--check-consistency", "1",
            "--fast-stat-sync", "--lr", "1e-3", "--bucket-cap-mb", "1", "--update-freq", "2", "--num-workers", "0",
            "--log-format", "simple", "--log-interval", "1"]
    cmds = [base + ["--distributed-gpus", "3", "--distributed-rank", "0"],
            base + ["--distributed-gpus", "5", "--distributed-rank", "3"]]
    out0, _ = _run_all(cmds, timeout=400)
    assert "(epoch 1 @ 3 updates)" in out0, out0[-2000:]
    # fast-stat sample size = seq_len x 8 ranks x update-freq 2 (reference bsz semantics, Q03)
    assert "bsz=512.000" in out0, out0[-2000:]
