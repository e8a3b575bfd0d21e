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


@pytest.fixture
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
