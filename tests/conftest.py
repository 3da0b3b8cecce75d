import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "3d-genome-cycle_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libgcs.so's HIP kernels)")


@pytest.fixture(scope="session")
def c1_design():
    from gcs import synthetic
    return synthetic.make_c1()


@pytest.fixture(scope="session")
def interphase_cfg():
    from gcs.config import InterphaseConfig
    return InterphaseConfig()
