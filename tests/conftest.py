import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libgcs.so's HIP kernels)")


def pytest_collection_modifyitems(config, items):
    if any(it.get_closest_marker("gpu") for it in items):
        # One HIP runtime per process: torch's device runtime is initialised BEFORE libgcs.so is loaded (the
        # engine loads it at its first construction), so the engine binds to that same runtime and shares device
        # pointers with torch tensors (gcs.domain's exchange buffers).  Loading libgcs.so first would start a
        # second runtime that torch then cannot use (tools/runtime_probe.py).
        import torch
        if torch.cuda.is_available():
            torch.zeros(1, device="cuda")


@pytest.fixture(scope="session")
def c1_design():
    from gcs import synthetic
    return synthetic.make_c1()


@pytest.fixture(scope="session")
def interphase_cfg():
    from gcs.config import InterphaseConfig
    return InterphaseConfig()
