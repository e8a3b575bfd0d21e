"""bench.py launch modes and the cross-rank-agreed native-comm fallback (CPU).

* ``python bench.py --gpus N`` without WORLD_SIZE starts N rank processes (env:// on
  127.0.0.1) and relays their exit status; ``--hetero 2,6`` starts one launch group per
  entry with the group's GPU count, device offset and a tcp:// rendezvous (BASELINE.json
  config 4, reference train.py:189-236); a ``--gpus`` that disagrees with an externally set
  WORLD_SIZE is refused.  The rank processes run the ``--dry-run`` hook: they report their
  environment and exit without touching a GPU.
* ``parallel.comm.create`` agrees across ranks before and after the RCCL rendezvous; a
  fault injected on one rank makes EVERY rank fall back to c10d with the reason recorded.
  Driven over gloo with a stand-in engine (two ranks of RCCL cannot share the one GPU of a
  test box).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, BENCH] + args, env=env, capture_output=True, text=True, timeout=120)
    ranks = [json.loads(line[len("DRYRUN "):]) for line in r.stdout.splitlines() if line.startswith("DRYRUN ")]
    return r.returncode, sorted(ranks, key=lambda d: int(d["RANK"] or 0)), r.stderr


def test_self_launch_starts_one_process_per_rank():
    rc, ranks, _ = _run(["--gpus", "3", "--dry-run", "-1"])
    assert rc == 0
    assert [d["RANK"] for d in ranks] == ["0", "1", "2"]
    assert [d["LOCAL_RANK"] for d in ranks] == ["0", "1", "2"]
    assert {d["WORLD_SIZE"] for d in ranks} == {"3"}
    assert len({d["MASTER_PORT"] for d in ranks}) == 1
    assert all(d["HETSEQ_INIT_METHOD"] is None for d in ranks)


def test_one_gpu_runs_in_process():
    rc, ranks, _ = _run(["--dry-run", "-1"])
    assert rc == 0 and len(ranks) == 1 and ranks[0]["RANK"] is None  # no launcher, no env


def test_failing_rank_fails_the_launch():
    rc, ranks, err = _run(["--gpus", "2", "--dry-run", "1"])
    assert rc != 0
    assert "rank process 1 exited" in err


def test_hetero_groups_map_ranks_and_devices():
    rc, ranks, _ = _run(["--hetero", "2,6", "--dry-run", "-1"])
    assert rc == 0 and len(ranks) == 8
    assert {d["WORLD_SIZE"] for d in ranks} == {"8"}
    init = {d["HETSEQ_INIT_METHOD"] for d in ranks}
    assert len(init) == 1 and init.pop().startswith("tcp://127.0.0.1:")
    g0 = [d for d in ranks if d["HETSEQ_GROUP"] == "0"]
    g1 = [d for d in ranks if d["HETSEQ_GROUP"] == "1"]
    assert [d["RANK"] for d in g0] == ["0", "1"] and [d["LOCAL_RANK"] for d in g0] == ["0", "1"]
    assert {d["HETSEQ_GROUP_GPUS"] for d in g0} == {"2"} and {d["HETSEQ_DEVICE_OFFSET"] for d in g0} == {"0"}
    assert [d["RANK"] for d in g1] == [str(r) for r in range(2, 8)]
    assert [d["LOCAL_RANK"] for d in g1] == [str(r) for r in range(6)]
    assert {d["HETSEQ_GROUP_GPUS"] for d in g1} == {"6"} and {d["HETSEQ_DEVICE_OFFSET"] for d in g1} == {"2"}
    # the device a rank drives = its group's offset + its local index = its global rank here
    from argparse import Namespace

    from hetseq_amd.parallel.distributed_utils import local_device_id

    for d in ranks:
        a = Namespace(device_id_offset=int(d["HETSEQ_DEVICE_OFFSET"]))
        assert local_device_id(a, int(d["LOCAL_RANK"])) == int(d["RANK"])


def test_gpus_must_match_world_size():
    rc, ranks, err = _run(["--gpus", "4", "--dry-run", "-1"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert rc == 2 and not ranks and "disagrees with WORLD_SIZE=2" in err
    rc, ranks, _ = _run(["--gpus", "2", "--dry-run", "-1"], {"WORLD_SIZE": "2", "RANK": "1"})
    assert rc == 0 and ranks[0]["RANK"] == "1"  # a torchrun-style rank runs in place
    rc, _, err = _run(["--gpus", "3", "--hetero", "2,6", "--dry-run", "-1"])
    assert rc == 2 and "disagrees with --hetero" in err


# ------------------------------------------------------------------ agreed native-comm fallback
def _fallback_worker(rank, world, path, fault, q):
    import torch
    import torch.distributed as dist

    from hetseq_amd.parallel import comm

    if fault:
        os.environ["HETSEQ_COMM_FAULT"] = fault
    dist.init_process_group("gloo", init_method="file://" + path, world_size=world, rank=rank)

    class FakeComm(object):
        """Stand-in engine: all-reduce through gloo, records that it was closed."""

        closed = None
        entered = False  # the (blocking) rendezvous was entered

        def __init__(self, group, timeout_s=0.0, rendezvous=True, key=None):
            self.group = group
            if rendezvous:
                self.rendezvous()

        def rendezvous(self):
            FakeComm.entered = True

        def all_reduce(self, t, op="sum", stream=None):
            dist.all_reduce(t, group=self.group)
            return t

        def check(self):
            pass

        def close(self, graceful=True):
            FakeComm.closed = graceful

    try:
        c = comm.create("native", False, factory=FakeComm)
        q.put((rank, c is not None, comm.LAST_STATUS, FakeComm.closed, FakeComm.entered))
    finally:
        dist.destroy_process_group()


def _fallback(tmp_path, fault, world=2):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fallback_worker, args=(r, world, str(tmp_path / "rdzv"), fault, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return out


@pytest.mark.slow
def test_init_fault_on_rank0_strands_nobody(tmp_path):
    """Rank 0 failing its local checks (it would have published the unique id) must not leave the
    other ranks waiting on the store: everyone agrees on the fallback within the call."""
    import time

    t0 = time.time()
    out = _fallback(tmp_path, "init:0", world=3)
    assert time.time() - t0 < 100
    assert [o[1] for o in out] == [False, False, False]
    assert "injected init fault on rank 0" in out[0][2]["reason"]
    assert not any(o[4] for o in out)


@pytest.mark.slow
def test_native_comm_used_when_every_rank_succeeds(tmp_path):
    out = _fallback(tmp_path, "")
    assert [o[1] for o in out] == [True, True]
    assert all(o[2] == {"engine": "rccl-native", "reason": None} for o in out)


@pytest.mark.slow
def test_init_fault_on_one_rank_falls_back_everywhere(tmp_path):
    out = _fallback(tmp_path, "init:1")
    assert [o[1] for o in out] == [False, False]  # nobody entered the rendezvous alone
    assert all(o[2]["engine"] == "c10d" for o in out)
    assert "injected init fault on rank 1" in out[1][2]["reason"]
    assert "another rank" in out[0][2]["reason"]
    assert not any(o[4] for o in out)  # nobody entered the rendezvous
    assert out[0][3] is False and out[1][3] is None  # rank 0 freed its local part (abort), rank 1 built none


@pytest.mark.slow
def test_bad_first_collective_aborts_on_every_rank(tmp_path):
    out = _fallback(tmp_path, "first:0")
    assert [o[1] for o in out] == [False, False]
    assert "first all-reduce returned" in out[0][2]["reason"]
    assert all(o[3] is False for o in out)  # every rank aborted (never a graceful, peer-waiting close)
    assert all(o[4] for o in out)  # after both entered the rendezvous
