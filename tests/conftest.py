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


@pytest.fixture(scope="session", autouse=True)
def _oracle_log_map_primitives():
    """On a GPU box, pin the oracle's log-MAP primitives (2^-t and log2 on their
    bounded grids, oracle/tdec_oracle.c orc_set_trans) to this device's
    v_exp_f32 / v_log_f32 outputs, so every log-MAP comparison is bit for bit;
    tests/test_gpu_logmap.py checks the tables are faithful (within 1 ulp of the
    correctly rounded values).  Without a GPU the oracle keeps the correctly
    rounded primitives."""
    try:
        import torch
        gpu = torch.cuda.is_available()
    except ImportError:
        gpu = False
    if not gpu:
        yield None
        return
    from modulations_amd import dvb_rcs2_turbo as M
    from oracle import oracle as O
    tabs = M.capture_trans_tables(0)
    O.set_trans(tabs)
    yield tabs
    O.set_trans(None)


@pytest.fixture(scope="session")
def trans_tables(_oracle_log_map_primitives):
    return _oracle_log_map_primitives
