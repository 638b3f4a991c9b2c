"""The C-ABI library builds, loads and exports every symbol include/tdec.h
declares; without a GPU it fails loudly (no host fallback)."""
import os
import re
import subprocess

import numpy as np
import pytest

from modulations_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "tdec.h")).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(tdec_\w+)\s*\(", src, re.M)))


def test_header_matches_binding_list():
    assert _header_symbols() == sorted(_native.EXPORTS)


def test_library_exports_every_symbol():
    lib = _native.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    for name in _header_symbols():
        assert re.search(rf"\bT {name}$", out, re.M), name
        assert hasattr(lib, name)


def test_library_is_gfx950():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data            # the embedded code object's target id


def test_no_silent_cpu_path_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from modulations_amd.dvb_rcs2_turbo import DVBRCS2_Turbo
    c = DVBRCS2_Turbo(48, "1/3")
    with pytest.raises(_native.TdecError):
        c.decode(np.zeros(c.n_coded))
