import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


_TORCH_READY = []


@pytest.fixture(autouse=True)
def _torch_before_library(request):
    """GPU tests: torch (its own HIP runtime) initialises the device before the product library's
    runtime does -- in the other order torch finds no GPU, and the partitioned tests hand torch
    tensors to the library."""
    if request.node.get_closest_marker("gpu") and not _TORCH_READY:
        _TORCH_READY.append(1)
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def hip_lib():
    """The product library; GPU tests fail loudly (no fallback) when it is missing."""
    from mcmc_colorer_amd import _lib

    return _lib.lib()
