import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the libsdiar kernels")


@pytest.fixture(scope="session")
def gpu():
    """GPU tests must run the native path: fail loudly if it is unavailable."""
    import torch
    from speaker_diarization_amd import _lib
    assert torch.cuda.is_available(), "gpu-marked test needs a HIP device"
    _lib.load()
    return torch.device("cuda", 0)
