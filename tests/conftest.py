"""pytest config: import paths, the `gpu` marker and shared fixtures."""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "openballbot-rl_amd", ROOT / "tests", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib

    oracle_lib.build()
    return oracle_lib


@pytest.fixture
def reward_config():
    return {"type": "directional", "config": {"target_direction": [0.0, 1.0]}}


@pytest.fixture
def terrain_config():
    return {"type": "flat", "config": {}}


@pytest.fixture
def test_state():
    return {"vel": np.array([0.5, 0.3, 0.0]), "orientation": np.array([0.1, 0.2, 0.3]),
            "pos2d": np.array([0.0, 0.0])}
