import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and the gfx950 library")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope="session")
def gpu():
    """The GPU tests fail (never skip) when the device or the HIP library is missing:
    a silent skip would hide a missing native path."""
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("pytest -m gpu needs a ROCm GPU (torch.cuda.is_available() is False)")
    from streamoptima_amd import _lib, build
    build.build()
    _lib.load()
    return torch.device("cuda:0")
