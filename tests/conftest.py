import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def golden(name):
    """Committed golden vectors (tests/golden/make_golden.py); plain arrays only."""
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def G_tables():
    return golden("tables")


@pytest.fixture(scope="session")
def G_siso():
    return golden("siso")


@pytest.fixture(scope="session")
def G_decode():
    return golden("decode")


@pytest.fixture(scope="session")
def G_encode():
    return golden("encode")


@pytest.fixture(scope="session")
def G_demap():
    return golden("demap")
