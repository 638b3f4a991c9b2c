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


@pytest.fixture(scope="session")
def _device_trans_tables():
    """This device's v_exp_f32 / v_log_f32 outputs on the log-MAP primitives'
    bounded grids (captured once per session), or None without a GPU."""
    try:
        import torch
        gpu = torch.cuda.is_available()
    except ImportError:
        gpu = False
    if not gpu:
        return None
    from modulations_amd import dvb_rcs2_turbo as M
    return M.capture_trans_tables(0)


@pytest.fixture(scope="module")
def trans_tables(_device_trans_tables):
    """Pin the oracle's log-MAP primitives (oracle/tdec_oracle.c orc_set_trans)
    to this device's instructions for the requesting module only, so its
    GPU-vs-oracle log-MAP comparisons are bit for bit; every other module
    (the CPU oracle tests included) sees the correctly rounded primitives
    whether or not the box has a GPU.  tests/test_gpu_logmap.py checks the
    tables are faithful (within 1 ulp of the correctly rounded values)."""
    from oracle import oracle as O
    if _device_trans_tables is not None:
        O.set_trans(_device_trans_tables)
    yield _device_trans_tables
    O.set_trans(None)
