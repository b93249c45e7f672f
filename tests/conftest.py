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


def _torch_first():
    """torch (its own HIP runtime) initialises the device before the product library is even
    loaded: with the library's HIP runtime loaded or initialised first, one of the two finds no
    GPU, and the partitioned tests hand torch tensors to the library."""
    if not _TORCH_READY:
        _TORCH_READY.append(1)
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()


_GPU_SESSION = []


def pytest_collection_modifyitems(config, items):
    if any(item.get_closest_marker("gpu") for item in items):
        _GPU_SESSION.append(1)


@pytest.fixture(scope="session", autouse=True)
def _torch_first_in_gpu_sessions():
    """A session that runs GPU tests initialises torch before any test (CPU ones included, e.g. the
    host CDF-walk hooks) loads the product library."""
    if _GPU_SESSION:
        _torch_first()
    yield


@pytest.fixture(autouse=True)
def _torch_before_library(request):
    if request.node.get_closest_marker("gpu"):
        _torch_first()
    yield


@pytest.fixture(scope="session")
def hip_lib():
    """The product library; GPU tests fail loudly (no fallback) when it is missing."""
    _torch_first()   # session fixtures are set up before the autouse one above
    from mcmc_colorer_amd import _lib

    return _lib.lib()
