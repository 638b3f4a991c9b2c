"""Soft-LLR demapper on MI355X: compute_llr of the reference harness
(test_sdr_with_coding.py:200-225) over the Gray constellations of the
reference (test_sdr_with_coding.py:25-100 for BPSK/QPSK/8PSK/16QAM,
sdr_modem.py:101-207 for 64QAM/256QAM).

``compute_llr(syms, mod_type, noise_var)`` returns exactly what the reference
returns (f64, positive for bit 1, clipped to +-30), including numpy's dtype
rules: the arithmetic is complex128 when the symbols or the constellation are
(QPSK's constellation is, because qpsk_mod divides by np.sqrt(2)), and the
final division stays float32 when noise_var ends up a Python float.
``sign=-1`` gives the decoder convention (positive for bit 0).
"""
from __future__ import annotations

import numpy as np

from . import _native as _n

GRAY2 = [0, 1, 3, 2]
GRAY3 = [0, 1, 3, 2, 6, 7, 5, 4]
GRAY4 = [0, 1, 3, 2, 6, 7, 5, 4, 12, 13, 15, 14, 10, 11, 9, 8]


# ---- mappers: same expressions (and so the same rounding) as the reference -------------
def bpsk_mod(bits):                                   # test_sdr_with_coding.py:25-26
    return 2.0 * np.array(bits, dtype=np.complex64) - 1.0


def qpsk_mod(bits):                                   # :31-37
    bits = np.array(bits)
    if len(bits) % 2:
        bits = np.append(bits, 0)
    I = 1 - 2 * bits[0::2]
    Q = 1 - 2 * bits[1::2]
    return (I + 1j * Q).astype(np.complex64) / np.sqrt(2)


def psk8_mod(bits):                                   # :45-57 (sdr_modem.py:120-130)
    bits = np.array(bits)
    pad = (3 - len(bits) % 3) % 3
    if pad:
        bits = np.append(bits, [0] * pad)
    b = bits.reshape(-1, 3)
    idx = b[:, 0] * 4 + b[:, 1] * 2 + b[:, 2]
    phase = np.array(GRAY3)[idx] * np.pi / 4
    return np.array([np.exp(1j * p) for p in phase], dtype=np.complex64)


def _qam_mod(bits, k, gray, scale):
    bits = np.array(bits)
    pad = (2 * k - len(bits) % (2 * k)) % (2 * k)
    if pad:
        bits = np.append(bits, [0] * pad)
    b = bits.reshape(-1, 2 * k)
    w = 1 << np.arange(k - 1, -1, -1)
    i_idx = b[:, :k] @ w
    q_idx = b[:, k:] @ w
    M = 1 << k
    syms = [((2 * gray[i] - (M - 1)) / np.sqrt(scale)) + 1j * ((2 * gray[q] - (M - 1)) / np.sqrt(scale))
            for i, q in zip(i_idx, q_idx)]
    return np.array(syms, dtype=np.complex64)


def qam16_mod(bits):                                  # :72-86 (sdr_modem.py:142-154)
    return _qam_mod(bits, 2, GRAY2, 10)


def qam64_mod(bits):                                  # sdr_modem.py:168-180
    return _qam_mod(bits, 3, GRAY3, 42)


def qam256_mod(bits):                                 # sdr_modem.py:195-207
    return _qam_mod(bits, 4, GRAY4, 170)


MODULATIONS = {
    'BPSK': {'mod': bpsk_mod, 'bps': 1, 'order': 2},
    'QPSK': {'mod': qpsk_mod, 'bps': 2, 'order': 4},
    '8PSK': {'mod': psk8_mod, 'bps': 3, 'order': 8},
    '16QAM': {'mod': qam16_mod, 'bps': 4, 'order': 16},
    '64QAM': {'mod': qam64_mod, 'bps': 6, 'order': 64},
    '256QAM': {'mod': qam256_mod, 'bps': 8, 'order': 256},
}


def constellation(mod_type):
    """Label-ordered constellation, exactly as compute_llr builds it (:207-208)."""
    m = MODULATIONS[mod_type]
    bps, order = m['bps'], m['order']
    all_bits = np.array([list(map(int, format(i, f'0{bps}b'))) for i in range(order)])
    return m['mod'](all_bits.flatten()).reshape(-1)


_CONS = {}


def _cons(mod_type):
    c = _CONS.get(mod_type)
    if c is None:
        c = _CONS[mod_type] = constellation(mod_type)
    return c


def demap_mode(syms_dtype, cons_dtype, noise_var):
    """(f64 arithmetic?, float32 division?, effective noise_var) by numpy's rules."""
    nv = max(noise_var, 0.005)                                     # :202
    f64 = np.result_type(syms_dtype, cons_dtype) == np.complex128
    div_f32 = (not f64) and (np.float32(1) / nv).dtype == np.float32
    return f64, div_f32, float(nv)


def compute_llr(syms, mod_type, noise_var, sign=+1, device=0):
    """Max-log soft demapper (reference test_sdr_with_coding.py:200-225) on the GPU."""
    m = MODULATIONS[mod_type]
    cons = _cons(mod_type)
    syms = np.asarray(syms)
    if syms.dtype not in (np.complex64, np.complex128):
        syms = syms.astype(np.complex128)
    syms = np.ascontiguousarray(syms)
    f64, div_f32, nv = demap_mode(syms.dtype, cons.dtype, noise_var)
    c = np.ascontiguousarray(cons.astype(np.complex128 if f64 else np.complex64))
    out = np.zeros(len(syms) * m['bps'])
    if len(syms):
        _n.check(_n.lib().tdec_demap(device, _n.ptr(syms), int(syms.dtype == np.complex128), len(syms),
                                     _n.ptr(c), int(f64), len(c), m['bps'], nv, int(div_f32), int(sign),
                                     _n.ptr(out)))
    return out


def compute_llr_device(syms, mod_type, noise_var, out=None, sign=+1, stream=None):
    """compute_llr over a device tensor of complex symbols (complex64/complex128 or
    a float [..., 2] view); returns a float64 device tensor."""
    import torch
    m = MODULATIONS[mod_type]
    cons = _cons(mod_type)
    sym_f64 = syms.dtype in (torch.complex128, torch.float64)
    n_sym = syms.numel() // (1 if syms.is_complex() else 2)
    f64, div_f32, nv = demap_mode(np.complex128 if sym_f64 else np.complex64, cons.dtype, noise_var)
    c = np.ascontiguousarray(cons.astype(np.complex128 if f64 else np.complex64))
    if syms.device.type != "cuda" or not syms.is_contiguous():
        raise ValueError("syms must be a contiguous tensor on a HIP device")
    if syms.dtype not in (torch.complex64, torch.complex128, torch.float32, torch.float64):
        raise TypeError(f"unsupported symbol dtype {syms.dtype}")
    dev = syms.device.index or 0
    if out is None:
        out = torch.empty(n_sym * m['bps'], dtype=torch.float64, device=syms.device)
    if out.dtype != torch.float64 or not out.is_contiguous() or out.numel() < n_sym * m['bps'] or out.device != syms.device:
        raise ValueError("out must be a contiguous float64 tensor of n_sym*bps elements on the symbols' device")
    st = _n.stream_ptr(stream) if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    _n.check(_n.lib().tdec_demap_dev(dev, _n.ptr(syms), int(sym_f64), n_sym, _n.ptr(c), int(f64),
                                     len(c), m['bps'], nv, int(div_f32), int(sign), _n.ptr(out), st))
    return out
