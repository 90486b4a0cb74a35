import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle as O  # tests/ may load the oracle (checker only)

    O.build()
    return O


@pytest.fixture(scope="session")
def orc(oracle_mod):
    return oracle_mod.Oracle()


def golden(name: str):
    import numpy as np

    return np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
