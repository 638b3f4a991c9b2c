"""ctypes bindings of the gfx950 HIP libraries (modulations_amd/lib/libtdec.so:
turbo decoder + soft demapper; modulations_amd/lib/libmodem.so: modem front-end).

The product path has no CPU fallback: if the library is missing or no HIP
device is visible, calls raise instead of computing anything on the host.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libtdec.so")
# A/B experiments only: TDEC_LIB_VARIANT=w4 loads lib/libtdec_w4.so (built by build.py --variant)
if os.environ.get("TDEC_LIB_VARIANT"):
    LIB_PATH = os.path.join(HERE, "lib", f"libtdec_{os.environ['TDEC_LIB_VARIANT']}.so")

TDEC_OK, TDEC_EINVAL, TDEC_ESHORT, TDEC_ENOMEM, TDEC_EHIP, TDEC_EUNSUPPORTED, TDEC_EITER, TDEC_ECAPACITY = \
    0, -1, -2, -3, -4, -5, -6, -7

# every symbol include/tdec.h declares (tests check the library exports them all)
EXPORTS = (
    "tdec_create", "tdec_destroy", "tdec_last_error", "tdec_llr_len", "tdec_siso_batch", "tdec_decode_batch",
    "tdec_reserve", "tdec_planes_bytes", "tdec_depuncture_dev", "tdec_decode_planes_dev", "tdec_decode_batch_dev",
    "tdec_tail_gate",
    "tdec_demap_dev", "tdec_demap", "tdec_demap_planes_dev", "tdec_encode_dev", "tdec_encoded_len",
    "tdec_demap_batch", "tdec_constellation", "tdec_workload_dev", "tdec_info_bits_dev", "tdec_count_errors_dev",
    "tdec_reserve_fused", "tdec_fused_available", "tdec_demap_decode_dev", "tdec_selftest", "tdec_selftest_trans",
    "tdec_host_alloc", "tdec_host_free", "tdec_encode_host", "tdec_siso_batch_f64", "tdec_siso_staging",
    "tdec_siso_staged", "tdec_siso_stats",
)

_lib = None
_lock = threading.Lock()

_vp = C.c_void_p


def _declare(L):
    L.tdec_create.argtypes = [C.c_int, C.c_int, C.c_int, _vp, C.c_int, C.c_int, _vp, _vp, _vp, C.POINTER(_vp)]
    L.tdec_create.restype = C.c_int
    L.tdec_destroy.argtypes = [_vp]
    L.tdec_destroy.restype = None
    L.tdec_last_error.argtypes = []
    L.tdec_last_error.restype = C.c_char_p
    L.tdec_llr_len.argtypes = [_vp]
    L.tdec_llr_len.restype = C.c_long
    L.tdec_encoded_len.argtypes = [_vp]
    L.tdec_encoded_len.restype = C.c_long
    L.tdec_siso_batch.argtypes = [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_double, _vp, _vp]
    if hasattr(L, "tdec_siso_batch_f64"):   # (A/B tools also load older builds without it)
        L.tdec_siso_batch_f64.argtypes = [_vp, C.c_int, _vp, _vp, _vp, _vp, _vp, _vp, C.c_double, _vp, _vp]
        L.tdec_siso_batch_f64.restype = C.c_int
        L.tdec_siso_staging.argtypes = [_vp, C.c_int, C.POINTER(_vp), C.POINTER(C.c_size_t)]
        L.tdec_siso_staging.restype = C.c_int
        L.tdec_siso_staged.argtypes = [_vp, C.c_int, C.c_int, C.c_double]
        L.tdec_siso_staged.restype = C.c_int
    if hasattr(L, "tdec_siso_stats"):
        L.tdec_siso_stats.argtypes = [_vp, C.POINTER(C.c_long)]
        L.tdec_siso_stats.restype = C.c_int
    L.tdec_decode_batch.argtypes = [_vp, C.c_int, _vp, C.c_long, _vp, _vp]
    L.tdec_reserve.argtypes = [_vp, C.c_int]
    L.tdec_planes_bytes.argtypes = [_vp, C.c_int]
    L.tdec_planes_bytes.restype = C.c_size_t
    L.tdec_depuncture_dev.argtypes = [_vp, C.c_int, _vp, C.c_long, _vp, _vp]
    L.tdec_decode_planes_dev.argtypes = [_vp, C.c_int, _vp, _vp, _vp, _vp]
    L.tdec_decode_batch_dev.argtypes = [_vp, C.c_int, _vp, C.c_long, _vp, _vp, _vp]
    if hasattr(L, "tdec_tail_gate"):   # (A/B tools also load older builds without it)
        L.tdec_tail_gate.argtypes = [_vp, _vp]
    L.tdec_demap_dev.argtypes = [C.c_int, _vp, C.c_int, C.c_long, _vp, C.c_int, C.c_int, C.c_int, C.c_double,
                                 C.c_int, C.c_int, _vp, _vp]
    L.tdec_demap.argtypes = [C.c_int, _vp, C.c_int, C.c_long, _vp, C.c_int, C.c_int, C.c_int, C.c_double,
                             C.c_int, C.c_int, _vp]
    L.tdec_demap_planes_dev.argtypes = [_vp, C.c_int, _vp, C.c_int, _vp, C.c_int, C.c_int, C.c_int, C.c_double,
                                        C.c_int, _vp, _vp]
    L.tdec_encode_dev.argtypes = [_vp, C.c_int, _vp, _vp, _vp]
    L.tdec_demap_batch.argtypes = [C.c_int, C.c_int, C.c_int, _vp, C.c_long, C.c_float, _vp]
    L.tdec_constellation.argtypes = [C.c_int, _vp, C.POINTER(C.c_int)]
    L.tdec_workload_dev.argtypes = [_vp, C.c_int, C.c_int64, C.c_uint64, _vp, C.c_int, C.c_int, C.c_double, _vp,
                                    _vp, _vp]
    L.tdec_info_bits_dev.argtypes = [_vp, C.c_int, C.c_int64, C.c_uint64, _vp, _vp]
    L.tdec_count_errors_dev.argtypes = [_vp, C.c_int, C.c_int64, C.c_uint64, _vp, _vp, _vp]
    L.tdec_reserve_fused.argtypes = [_vp, C.c_int]
    L.tdec_fused_available.argtypes = [_vp, C.c_int, C.c_int]
    L.tdec_demap_decode_dev.argtypes = [_vp, C.c_int, _vp, C.c_int, _vp, C.c_int, C.c_int, C.c_int, C.c_double,
                                        C.c_int, _vp, _vp, _vp]
    L.tdec_selftest.argtypes = [C.c_int, C.c_int, C.c_longlong, C.c_ulonglong, C.POINTER(C.c_longlong)]
    L.tdec_selftest_trans.argtypes = [C.c_int, C.c_int, C.c_uint32, C.c_longlong, _vp]
    L.tdec_host_alloc.argtypes = [C.c_size_t, C.POINTER(_vp)]
    L.tdec_host_free.argtypes = [_vp]
    L.tdec_host_free.restype = None
    if hasattr(L, "tdec_encode_host"):   # (A/B tools also load older builds without it)
        L.tdec_encode_host.argtypes = [C.c_int, C.c_int, _vp, _vp, C.c_long, _vp, C.c_long, _vp, C.c_long]
        L.tdec_encode_host.restype = C.c_long
    for name in EXPORTS:
        if not hasattr(L, name):
            continue
        f = getattr(L, name)
        if f.restype is C.c_int or name in ("tdec_siso_batch", "tdec_decode_batch", "tdec_reserve",
                                            "tdec_depuncture_dev", "tdec_decode_planes_dev",
                                            "tdec_decode_batch_dev", "tdec_demap_dev", "tdec_demap",
                                            "tdec_demap_planes_dev", "tdec_encode_dev", "tdec_demap_batch",
                                            "tdec_constellation", "tdec_workload_dev", "tdec_info_bits_dev",
                                            "tdec_count_errors_dev", "tdec_reserve_fused", "tdec_fused_available",
                                            "tdec_demap_decode_dev", "tdec_selftest", "tdec_selftest_trans",
                                            "tdec_host_alloc"):
            f.restype = C.c_int


def lib():
    """Load libtdec.so (building it first if this is a build tree without it)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    from . import build
                    build.build()
                L = C.CDLL(LIB_PATH)
                _declare(L)
                _lib = L
    return _lib


class TdecError(RuntimeError):
    pass


def check(rc):
    if rc == TDEC_OK:
        return
    msg = lib().tdec_last_error().decode(errors="replace")
    if rc == TDEC_EINVAL or rc == TDEC_EUNSUPPORTED:
        raise ValueError(msg)
    if rc == TDEC_ESHORT:
        raise IndexError(msg)
    if rc == TDEC_ENOMEM:
        raise MemoryError(msg)
    if rc == TDEC_EITER:
        raise UnboundLocalError(msg)
    raise TdecError(f"tdec error {rc}: {msg}")


def ptr(a):
    """Device or host address of a numpy array / torch tensor (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


def stream_ptr(stream):
    if stream is None:
        return None
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


# ---------------------------------------------------------------- libmodem.so ----------
MODEM_LIB_PATH = os.path.join(HERE, "lib", "libmodem.so")
MDM_ENAN = -8
# every symbol include/modem.h declares
MODEM_EXPORTS = (
    "mdm_map_dev", "mdm_map", "mdm_demod_dev", "mdm_demod", "mdm_fir_dev", "mdm_fir",
    "mdm_iq_quantize_dev", "mdm_iq_quantize", "mdm_iq_dequantize_dev", "mdm_iq_dequantize", "mdm_last_error",
)
_mlib = None


def _declare_modem(L):
    i, l, d = C.c_int, C.c_long, C.c_double
    L.mdm_map_dev.argtypes = [i, _vp, l, i, _vp, i, _vp, _vp]
    L.mdm_map.argtypes = [i, _vp, l, i, _vp, i, _vp]
    L.mdm_demod_dev.argtypes = [i, i, _vp, i, l, i, _vp, d, _vp, i, _vp, _vp, _vp]
    L.mdm_demod.argtypes = [i, i, _vp, i, l, i, _vp, d, _vp, i, _vp]
    L.mdm_fir_dev.argtypes = [i, _vp, i, l, _vp, i, i, i, l, l, _vp, _vp]
    L.mdm_fir.argtypes = [i, _vp, i, l, _vp, i, i, i, l, l, _vp]
    L.mdm_iq_quantize_dev.argtypes = [i, _vp, i, l, _vp, _vp, _vp]
    L.mdm_iq_quantize.argtypes = [i, _vp, i, l, _vp]
    L.mdm_iq_dequantize_dev.argtypes = [i, _vp, l, _vp, _vp]
    L.mdm_iq_dequantize.argtypes = [i, _vp, l, _vp]
    for name in MODEM_EXPORTS:
        getattr(L, name).restype = C.c_int
    L.mdm_last_error.argtypes = []
    L.mdm_last_error.restype = C.c_char_p


def modem_lib():
    """Load libmodem.so (building it first if this is a build tree without it)."""
    global _mlib
    if _mlib is None:
        with _lock:
            if _mlib is None:
                if not os.path.exists(MODEM_LIB_PATH):
                    from . import build
                    build.build_modem()
                L = C.CDLL(MODEM_LIB_PATH)
                _declare_modem(L)
                _mlib = L
    return _mlib


def modem_check(rc):
    if rc == TDEC_OK:
        return
    msg = modem_lib().mdm_last_error().decode(errors="replace")
    if rc in (TDEC_EINVAL, MDM_ENAN):
        raise ValueError(msg)
    if rc == TDEC_ENOMEM:
        raise MemoryError(msg)
    raise TdecError(f"modem error {rc}: {msg}")
