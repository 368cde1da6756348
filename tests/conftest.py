import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_built():
    # Build the in-tree extension once per session (no-op when fresh).
    from alluxio_amd.ops.native import lib
    lib()
    yield


@pytest.fixture
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test ran without a visible HIP device")
    return torch.device("cuda", 0)
