import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


@pytest.fixture(scope="session")
def states():
    return dict(np.load(os.path.join(HERE, "golden", "states.npz"), allow_pickle=False))


@pytest.fixture(scope="session")
def oracle_golden():
    return dict(np.load(os.path.join(HERE, "golden", "oracle.npz"), allow_pickle=False))


def state_key(L, p, N, J, U):
    return f"L{L}_p{p}_N{N}_J{J:g}_U{U:g}"
