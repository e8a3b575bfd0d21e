import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    """Build the in-tree extensions once per session (no-op when up to date)."""
    from hetseq_amd.csrc import build

    build.build_native()
    build.build_h5()
    try:
        import torch

        if torch.cuda.is_available():
            build.build_hip()
            build.build_comm()
    except Exception:
        pass
    yield


_STREAMS_DEFAULT = None


@pytest.fixture(autouse=True)
def _isolate_process_state():
    """No process-global runtime state leaks from one test into the next: TunableOp (a live
    library tuning pass once faulted a later test's reference GEMM), the measured GEMM engine
    choices, the weight-gradient side-stream switch, the device-seed pointer of the dropout
    kernels and the fp32 product engine."""
    global _STREAMS_DEFAULT
    from hetseq_amd.runtime import streams

    if _STREAMS_DEFAULT is None:
        _STREAMS_DEFAULT = streams._ENABLED
    yield
    import torch

    from hetseq_amd.ops import gemm as G
    from hetseq_amd.runtime import gemm_tuning, rng

    gemm_tuning.reset()
    G.GEMM_CHOICES.clear()
    if G.fp32_mode() != G.FP32_DEFAULT:
        G.set_fp32_mode(G.FP32_DEFAULT)
    streams.set_enabled(_STREAMS_DEFAULT)
    if torch.cuda.is_available():
        rng.disable_device_seed()
        torch.cuda.synchronize()


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
