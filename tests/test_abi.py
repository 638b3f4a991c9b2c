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


def test_builtin_constellations_match_the_mapper_tables():
    """tdec_constellation (host only) rebuilds the label-ordered tables that
    compute_llr gets from the reference mappers, value and dtype exact."""
    import ctypes as C
    import numpy as np
    from modulations_amd import demap as D
    L = _native.lib()
    for mod_id, name in enumerate(("BPSK", "QPSK", "8PSK", "16QAM", "64QAM", "256QAM")):
        iq = np.zeros(512)
        f64 = C.c_int(-1)
        M = L.tdec_constellation(mod_id, _native.ptr(iq), C.byref(f64))
        want = D.constellation(name)
        assert M == len(want), name
        assert bool(f64.value) == (want.dtype == np.complex128), name
        got = iq[0:2 * M:2] + 1j * iq[1:2 * M:2]
        assert np.array_equal(got, want.astype(np.complex128)), name
    assert L.tdec_constellation(6, _native.ptr(np.zeros(512)), C.byref(C.c_int())) == _native.TDEC_EINVAL


def test_build_record_identifies_the_loaded_library():
    """lib/*.build.json (written by modulations_amd.build) names the binary and the
    source digest that profiles/traffic.json measurements are keyed by."""
    import hashlib
    from modulations_amd import build as B
    for out, deps in ((B.OUT, B.DEPS), (B.MODEM_OUT, B.MODEM_DEPS)):
        info = B.build_info(out)
        if info is None:
            pytest.skip("library built without a build record")
        with open(out, "rb") as f:
            assert info["lib_sha256"] == hashlib.sha256(f.read()).hexdigest()
        assert info["src_sha256"] == B.source_digest(deps)
