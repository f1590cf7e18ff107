"""Shared test setup.  `-m "not gpu"` runs on the CPU-only build container; `-m gpu` on MI355X."""
from __future__ import annotations

import glob
import importlib
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")


def load_pkg():
    """The product package (its directory name starts with a digit, so import by string)."""
    return importlib.import_module("3dgaussian_amd")


def golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz")) as d:
        return {k: d[k] for k in d.files}


def golden_names(prefix: str):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


@pytest.fixture(scope="session")
def pkg():
    return load_pkg()


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _fresh_lazy_depth():
    """Every test starts with the drop-in op's adaptive laziness unlearned (torch_renderer.reset_lazy_depth)."""
    mod = sys.modules.get("3dgaussian_amd.torch_renderer")
    if mod is not None:
        mod.reset_lazy_depth()
    yield
