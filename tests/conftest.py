import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "python-audio-tools_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session", autouse=True)
def _torch_first(request):
    """torch's HIP runtime must come up before libatgpu's in a GPU run
    (tests hand torch device buffers to the library, and torch cannot
    initialise once libatgpu's runtime has), whatever test runs first"""
    if request.config.getoption("-m") and "not gpu" in request.config.getoption("-m"):
        return
    try:
        import torch
    except ImportError:
        return
    if torch.cuda.is_available():
        torch.cuda.init()


@pytest.fixture(scope="session")
def gpu_engine():
    # torch's HIP runtime comes up first: tests hand torch device buffers to
    # the engine, and torch cannot initialise once libatgpu's runtime has
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from audiotools import _atgpu
    return _atgpu.engine()
