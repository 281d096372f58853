import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mxk8s.ops import _lib
    _lib.lib()   # fail loudly if the HIP library is missing on a GPU box
    return torch.device("cuda", 0)


@pytest.fixture
def fixtures_dir():
    return os.path.join(REPO, "tests", "fixtures")
