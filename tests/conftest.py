import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built hipserve/_C.so")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    markexpr = config.getoption("-m") or ""
    if _gpu_available():
        return
    # On a CPU-only host, GPU tests are skipped unless explicitly selected with -m gpu
    # (then they fail loudly, which is what we want on a GPU box that lost its GPU).
    if "gpu" in markexpr and "not gpu" not in markexpr:
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
