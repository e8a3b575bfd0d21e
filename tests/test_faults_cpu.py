"""Failure handling: a rank that dies mid-training must turn into a
bounded-time error on its peers (collective timeout / broken connection), never
a hang; an injected exception propagates.  gloo, 2 processes, CPU."""
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mnist_dir(tmp_path):
    from hetseq_amd.data.synthetic import write_mnist

    d = tmp_path / "mnist"
    write_mnist(str(d), n_train=256, n_test=64, seed=3)
    return str(d)


def _launch(tmp_path, data, rank, port, fault, timeout_s):
    env = dict(os.environ, HETSEQ_FAULT=fault, PYTHONPATH=ROOT)
    cmd = [sys.executable, os.path.join(ROOT, "train.py"), "--task", "mnist", "--optimizer", "adadelta", "--lr", "1.0",
           "--data", data, "--max-sentences", "16", "--valid-subset", "test", "--cpu", "--max-epoch", "3",
           "--log-format", "none", "--distributed-backend", "gloo",
           "--distributed-world-size", "2", "--distributed-rank", str(rank), "--distributed-gpus", "1",
           "--distributed-init-method", "tcp://127.0.0.1:%d" % port, "--collective-timeout", str(timeout_s),
           "--save-dir", str(tmp_path / ("ck%d" % rank)), "--no-save", "--fast-stat-sync"]
    return subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def test_killed_rank_fails_peer_in_bounded_time(tmp_path):
    data = _mnist_dir(tmp_path)
    port = _free_port()
    t0 = time.time()
    procs = [_launch(tmp_path, data, r, port, "kill:1@3", 20) for r in range(2)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    elapsed = time.time() - t0
    assert procs[1].returncode == 17, outs[1][-2000:]
    assert procs[0].returncode != 0, outs[0][-2000:]  # the survivor errors out instead of hanging
    assert elapsed < 200


def test_injected_exception_propagates(tmp_path):
    data = _mnist_dir(tmp_path)
    port = _free_port()
    procs = [_launch(tmp_path, data, r, port, "raise:0@2", 20) for r in range(2)]
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert procs[0].returncode != 0 and "InjectedFault" in outs[0], outs[0][-2000:]
    assert procs[1].returncode != 0, outs[1][-2000:]
