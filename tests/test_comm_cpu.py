"""Native RCCL engine: build, rendezvous id and engine selection (CPU; the collectives run in
tests/test_comm_gpu.py on an MI355X)."""
import warnings

import pytest
import torch
import torch.distributed as dist


def test_module_builds_and_draws_unique_ids():
    from hetseq_amd.csrc import build
    from hetseq_amd.parallel import comm

    build.build_comm()
    mod = comm.module()
    assert mod is not None
    a, b = mod.unique_id(), mod.unique_id()
    assert len(a) == 128 and a != b
    assert mod.rccl_version() >= 22000


def test_engine_selection_on_gloo(tmp_path):
    from hetseq_amd.parallel import comm

    dist.init_process_group("gloo", init_method="file://" + str(tmp_path / "rdzv"), world_size=1, rank=0)
    try:
        assert comm.create("auto", False) is None  # CPU tensors: c10d / gloo
        assert comm.create("c10d", True) is None
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            assert comm.create("native", True) is None  # gloo backend: native needs RCCL
        assert any("nccl" in str(x.message) for x in w)
    finally:
        dist.destroy_process_group()


def test_flatddp_cpu_keeps_c10d(tmp_path):
    from hetseq_amd.parallel.ddp import FlatDDP
    from hetseq_amd.runtime.flat import FlatParamStore

    dist.init_process_group("gloo", init_method="file://" + str(tmp_path / "rdzv"), world_size=1, rank=0)
    try:
        net = torch.nn.Linear(4, 3)
        store = FlatParamStore(net)
        ddp = FlatDDP(net, store, comm_engine="auto")
        assert ddp.comm is None
        ddp(torch.randn(2, 4)).sum().backward()
        s = torch.ones(6, dtype=torch.float64)
        assert torch.equal(ddp.all_reduce_(s), torch.ones(6, dtype=torch.float64))
    finally:
        dist.destroy_process_group()
