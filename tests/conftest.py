"""Shared fixtures. `-m gpu` tests need a visible MI355X; `-m "not gpu"` tests run anywhere."""
import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: takes more than a few seconds")


@pytest.fixture(scope="session")
def golden_meta():
    return json.loads((GOLD / "golden.json").read_text())


def load_npz(name):
    with np.load(GOLD / name, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def crt():
    import cpp_raytracer_amd
    return cpp_raytracer_amd
