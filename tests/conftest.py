import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multimodal-embedding_amd"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libmme)")
    config.addinivalue_line("markers", "slow: full-size case (minutes)")
    config.addinivalue_line("markers", "dev: exercises a development kernel form (needs libmme_dev.so, MME_DEV=1)")


def pytest_collection_modifyitems(config, items):
    """`dev` tests run against the development library only (MME_DEV=1); the production
    libmme.so holds the dispatched kernels alone."""
    if os.environ.get("MME_DEV", "0") == "1":
        return
    skip = pytest.mark.skip(reason="development kernel form: run with MME_DEV=1 (make dev)")
    for it in items:
        if "dev" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"))
    return load


@pytest.fixture(scope="session")
def cuda():
    import torch
    assert torch.cuda.is_available(), "gpu-marked test needs a visible MI355X (no CPU fallback exists)"
    from mme import _lib
    _lib.load()
    return torch.device("cuda")
