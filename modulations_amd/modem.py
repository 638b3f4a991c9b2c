"""Modem front-end on MI355X: the reference's symbol
mappers, hard-decision demodulators, RRC pulse shaping / matched filtering
and int8/uint8 IQ sample format, behind the reference's own names.

  SDRModem            sdr_modem.py:17-342 (the modem part: mappers, demods,
                      _rrc_filter, _upsample_filter, modulate/demodulate,
                      _save_iq/_load_iq; radio I/O, sync and carrier recovery
                      are out of scope)
  Modulator,          modulators.py:19-199 (natural-label mappers, argmin QAM
  rrcosfilter         demods, upfirdn pulse shaping, matched filter)
  bpsk_mod ...        test_sdr_with_coding.py:25-128, 228-240 (the harness
  rrc_taps, ...       copies: mappers/demods, rrc_taps, upsample_filter,
  save_iq, load_iq    save_iq, load_iq)

Host work is limited to setup the reference also does once per call or per
object -- constellation tables, label maps and filter taps, built with the
reference's own numpy expressions -- and file I/O.  Every per-symbol and
per-sample operation runs in libmodem.so (include/modem.h) on the GPU; there
is no CPU fallback.  Outputs keep the reference's dtypes (int64 bits,
complex64/complex128 symbols, complex128 filter outputs).

Deliberate deviations, all documented in DESIGN.md §3: bits must be 0/1 (the
reference's integer arithmetic on other values has no table form); the
int8 conversion of _save_iq takes complex input (a real array is treated as
complex with zero imaginary part, which numpy would divide without Smith's
method); SDRModem.sync_syms is computed on first use instead of in __init__.
"""
from __future__ import annotations

import numpy as np

from . import _native as _n
from . import demap as D

# ---------------------------------------------------------------- C-ABI wrappers ------------
GT0, QPSK, PSK8, QAM_AXIS, ARGMIN = 0, 1, 2, 3, 4


def _bits_u8(bits):
    b = np.asarray(bits)
    if b.dtype == np.uint8 and b.flags.c_contiguous:
        u = b.ravel()
    else:
        u = np.ascontiguousarray(b.ravel())
        if u.size and not np.all((u == 0) | (u == 1)):
            raise ValueError("bits must be 0 or 1")
        u = u.astype(np.uint8)
    if u.size and u.max(initial=0) > 1:
        raise ValueError("bits must be 0 or 1")
    return u


def map_bits(bits, bps, table, device=0):
    """Labels (MSB first, zero-padded to whole symbols) -> table[label] on the GPU."""
    table = np.ascontiguousarray(table)
    assert table.dtype in (np.complex64, np.complex128) and table.size == 1 << bps
    u = _bits_u8(bits)
    n_sym = -(-u.size // bps)
    out = np.empty(n_sym, table.dtype)
    if u.size:
        _n.modem_check(_n.modem_lib().mdm_map(device, _n.ptr(u), u.size, bps, _n.ptr(table),
                                              int(table.dtype == np.complex128), _n.ptr(out)))
    return out


def _syms_c(syms):
    s = np.asarray(syms)
    if s.dtype not in (np.complex64, np.complex128):
        s = s.astype(np.complex128)
    return np.ascontiguousarray(s.ravel())


def hard_demod(syms, kind, bps, labels=None, scale=0.0, cons=None, nan_raises=True, device=0):
    """uint8 bits [n_sym * bps] of the given rule (include/modem.h MDM_DEMOD_*)."""
    s = _syms_c(syms)
    out = np.empty(s.size * bps, np.uint8)
    lab = None if labels is None else np.ascontiguousarray(labels, np.int32)
    c = None if cons is None else np.ascontiguousarray(cons, np.complex128)
    if s.size:
        _n.modem_check(_n.modem_lib().mdm_demod(device, kind, _n.ptr(s), int(s.dtype == np.complex128), s.size, bps,
                                                _n.ptr(lab), float(scale), _n.ptr(c), int(bool(nan_raises)),
                                                _n.ptr(out)))
    return out


def fir(x, taps, up=1, down=1, offset=0, n_out=None, device=0):
    """out[i] = sum_k taps[k] * xu[i*down + offset - k] (complex128), see modem.h."""
    s = _syms_c(x)
    h = np.ascontiguousarray(taps, np.float64)
    out = np.empty(n_out, np.complex128)
    if n_out:
        _n.modem_check(_n.modem_lib().mdm_fir(device, _n.ptr(s), int(s.dtype == np.complex128), s.size, _n.ptr(h),
                                              h.size, up, down, offset, n_out, _n.ptr(out)))
    return out


def iq_quantize(sig, device=0):
    """_save_iq's int8 interleaved samples of a complex signal."""
    s = np.asarray(sig)
    if s.dtype not in (np.complex64, np.complex128):
        s = s.astype(np.complex128)
    s = np.ascontiguousarray(s.ravel())
    if s.size == 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    out = np.empty(2 * s.size, np.int8)
    _n.modem_check(_n.modem_lib().mdm_iq_quantize(device, _n.ptr(s), int(s.dtype == np.complex128), s.size,
                                                  _n.ptr(out)))
    return out


def iq_dequantize(raw, device=0):
    """_load_iq's complex64 samples of interleaved uint8 I/Q bytes."""
    r = np.ascontiguousarray(np.asarray(raw, np.uint8).ravel())
    if r.size % 2:
        # raw[0::2] has one sample more than raw[1::2]: I + 1j * Q broadcasts
        # only when Q has 0 or 1 samples, as numpy does
        if r.size == 1:
            return np.zeros(0, np.complex64)
        if r.size == 3:
            r = np.array([r[0], r[1], r[2], r[1]], np.uint8)
        else:
            raise ValueError(f"operands could not be broadcast together with shapes ({r.size // 2 + 1},) "
                             f"({r.size // 2},)")
    out = np.empty(r.size // 2, np.complex64)
    if out.size:
        _n.modem_check(_n.modem_lib().mdm_iq_dequantize(device, _n.ptr(r), out.size, _n.ptr(out)))
    return out


# ---- device-resident forms (torch tensors on the GPU, stream-ordered) ----------------------
def map_device(bits, bps, table, out=None, stream=None):
    import torch
    table = np.ascontiguousarray(table)
    f64 = table.dtype == np.complex128
    n_sym = -(-bits.numel() // bps)
    if out is None:
        out = torch.empty(n_sym, dtype=torch.complex128 if f64 else torch.complex64, device=bits.device)
    _n.modem_check(_n.modem_lib().mdm_map_dev(bits.device.index or 0, _n.ptr(bits), bits.numel(), bps, _n.ptr(table),
                                              int(f64), _n.ptr(out), _n.stream_ptr(stream)))
    return out


def demod_device(syms, kind, bps, labels=None, scale=0.0, cons=None, nan_raises=True, out=None, nan_count=None,
                 stream=None):
    import torch
    lab = None if labels is None else np.ascontiguousarray(labels, np.int32)
    c = None if cons is None else np.ascontiguousarray(cons, np.complex128)
    if out is None:
        out = torch.empty(syms.numel() * bps, dtype=torch.uint8, device=syms.device)
    _n.modem_check(_n.modem_lib().mdm_demod_dev(syms.device.index or 0, kind, _n.ptr(syms),
                                                int(syms.dtype == torch.complex128), syms.numel(), bps, _n.ptr(lab),
                                                float(scale), _n.ptr(c), int(bool(nan_raises)), _n.ptr(out),
                                                _n.ptr(nan_count), _n.stream_ptr(stream)))
    return out


def fir_device(x, taps, up=1, down=1, offset=0, n_out=None, out=None, stream=None):
    import torch
    h = np.ascontiguousarray(taps, np.float64)
    if out is None:
        out = torch.empty(n_out, dtype=torch.complex128, device=x.device)
    _n.modem_check(_n.modem_lib().mdm_fir_dev(x.device.index or 0, _n.ptr(x), int(x.dtype == torch.complex128),
                                              x.numel(), _n.ptr(h), h.size, up, down, offset, n_out, _n.ptr(out),
                                              _n.stream_ptr(stream)))
    return out


def iq_quantize_device(sig, out=None, scratch=None, stream=None):
    import torch
    if out is None:
        out = torch.empty(2 * sig.numel(), dtype=torch.int8, device=sig.device)
    if scratch is None:
        scratch = torch.empty(1, dtype=torch.int64, device=sig.device)
    _n.modem_check(_n.modem_lib().mdm_iq_quantize_dev(sig.device.index or 0, _n.ptr(sig),
                                                      int(sig.dtype == torch.complex128), sig.numel(), _n.ptr(out),
                                                      _n.ptr(scratch), _n.stream_ptr(stream)))
    return out


def iq_dequantize_device(raw, out=None, stream=None):
    import torch
    n = raw.numel() // 2
    if out is None:
        out = torch.empty(n, dtype=torch.complex64, device=raw.device)
    _n.modem_check(_n.modem_lib().mdm_iq_dequantize_dev(raw.device.index or 0, _n.ptr(raw), n, _n.ptr(out),
                                                        _n.stream_ptr(stream)))
    return out


# ---------------------------------------------------------------- filter design (host) --------
def _rrc_taps(sps, alpha=0.35, ntaps=101):
    """sdr_modem.py:77-91 / test_sdr_with_coding.py:110-123: the same scalar
    expressions per tap (so the same rounding), normalised by np.linalg.norm."""
    h = np.zeros(ntaps)
    offs = np.arange(ntaps) - (ntaps - 1) / 2
    for i, t in enumerate(offs / sps):
        if t == 0:
            h[i] = 1 - alpha + 4 * alpha / np.pi
            continue
        if abs(abs(t) - 1 / (4 * alpha)) < 1e-8:
            h[i] = alpha / np.sqrt(2) * ((1 + 2 / np.pi) * np.sin(np.pi / 4 / alpha) +
                                         (1 - 2 / np.pi) * np.cos(np.pi / 4 / alpha))
            continue
        den = np.pi * t * (1 - (4 * alpha * t) ** 2)
        if abs(den) > 1e-8:
            h[i] = (np.sin(np.pi * t * (1 - alpha)) + 4 * alpha * t * np.cos(np.pi * t * (1 + alpha))) / den
    return h / np.linalg.norm(h)


def rrc_taps(sps, alpha=0.35, ntaps=101):
    """test_sdr_with_coding.py:110-123."""
    return _rrc_taps(sps, alpha, ntaps)


def rrcosfilter(N, alpha, Ts, Fs):
    """modulators.py:19-47: int(N*Fs)|1 taps, the same per-tap expressions,
    normalised by sqrt(sum(h**2))."""
    n = int(N * Fs) | 1
    t_all = (np.arange(n) - (n - 1) / 2) * (1.0 / float(Fs))
    h = np.zeros(len(t_all), dtype=float)
    for i in range(n):
        t = t_all[i]
        if t == 0.0:
            h[i] = 1.0 - alpha + (4 * alpha / np.pi)
        elif alpha != 0 and abs(t) == Ts / (4 * alpha):
            h[i] = (alpha / np.sqrt(2)) * (((1 + 2 / np.pi) * (np.sin(np.pi / (4 * alpha)))) +
                                           ((1 - 2 / np.pi) * (np.cos(np.pi / (4 * alpha)))))
        else:
            den = 1 - (4 * alpha * t / Ts) ** 2
            if abs(den) < 1e-10:
                den = 1e-10
            h[i] = (np.sin(np.pi * t / Ts * (1 - alpha)) + 4 * alpha * t / Ts * np.cos(np.pi * t / Ts * (1 + alpha))) \
                / (np.pi * t / Ts * den)
    return h / np.sqrt(np.sum(h ** 2))


def _same_conv_up(syms, sps, taps, device):
    """np.convolve(up, taps, 'same') with up = zeros(len*sps, complex64), up[::sps] = syms."""
    s = np.asarray(syms)
    n_up = len(s) * sps
    if n_up == 0:
        raise ValueError("a cannot be empty")
    s = np.ascontiguousarray(s.astype(np.complex64).ravel())
    L = len(taps)
    return fir(s, taps, up=sps, down=1, offset=(min(n_up, L) - 1) // 2, n_out=max(n_up, L), device=device)


def upsample_filter(syms, sps, taps, device=0):
    """test_sdr_with_coding.py:125-128."""
    return _same_conv_up(syms, sps, taps, device)


# ---------------------------------------------------------------- IQ files ------------------
def save_iq(sig, fname, device=0):
    """test_sdr_with_coding.py:228-233 / sdr_modem.py:329-335."""
    iq_quantize(sig, device).tofile(fname)


def load_iq(fname, device=0):
    """test_sdr_with_coding.py:235-240 / sdr_modem.py:337-342."""
    return iq_dequantize(np.fromfile(fname, dtype=np.uint8), device)


# ---------------------------------------------------------------- Gray family ---------------
GRAY2, GRAY3, GRAY4 = D.GRAY2, D.GRAY3, D.GRAY4
_INV = {k: [g.index(i) for i in range(len(g))] for k, g in ((2, GRAY2), (3, GRAY3), (4, GRAY4))}

_TABLES = {}


def _gray_table(mod):
    t = _TABLES.get(("gray", mod))
    if t is None:
        t = _TABLES[("gray", mod)] = D.constellation(mod)   # the reference mappers over every label
    return t


def _loop_bits(bits):
    """np.array(list of Python ints) of the reference's per-symbol loops: int64,
    or float64 when empty."""
    return bits.astype(np.int64) if bits.size else np.array([])


def bpsk_mod(bits, device=0):
    """test_sdr_with_coding.py:25-26 / sdr_modem.py:101-102 (1 -> +1, 0 -> -1)."""
    return map_bits(bits, 1, _gray_table("BPSK"), device)


def bpsk_demod(syms, device=0):
    """test_sdr_with_coding.py:28-29 / sdr_modem.py:104-105."""
    return hard_demod(syms, GT0, 1, device=device).astype(int)


def qpsk_mod(bits, device=0):
    """test_sdr_with_coding.py:31-37 / sdr_modem.py:107-112 (complex128)."""
    return map_bits(bits, 2, _gray_table("QPSK"), device)


def qpsk_demod(syms, device=0):
    """test_sdr_with_coding.py:39-43 / sdr_modem.py:114-118."""
    return hard_demod(syms, QPSK, 2, device=device).astype(int)


def psk8_mod(bits, device=0):
    """test_sdr_with_coding.py:45-57 / sdr_modem.py:120-130."""
    return map_bits(bits, 3, _gray_table("8PSK"), device)


def psk8_demod(syms, device=0):
    """test_sdr_with_coding.py:59-70 / sdr_modem.py:132-140 (int(NaN) raises)."""
    return _loop_bits(hard_demod(syms, PSK8, 3, labels=_INV[3], nan_raises=True, device=device))


def _qam_demod(syms, k, scale, device):
    return _loop_bits(hard_demod(syms, QAM_AXIS, 2 * k, labels=_INV[k], scale=scale, device=device))


def qam16_mod(bits, device=0):
    """test_sdr_with_coding.py:72-86 / sdr_modem.py:142-154."""
    return map_bits(bits, 4, _gray_table("16QAM"), device)


def qam16_demod(syms, device=0):
    """test_sdr_with_coding.py:88-100 / sdr_modem.py:156-166."""
    return _qam_demod(syms, 2, np.sqrt(10), device)


MODULATIONS = {
    'BPSK': {'mod': bpsk_mod, 'demod': bpsk_demod, 'bps': 1, 'order': 2, 'alpha': 0.02},
    'QPSK': {'mod': qpsk_mod, 'demod': qpsk_demod, 'bps': 2, 'order': 4, 'alpha': 0.015},
    '8PSK': {'mod': psk8_mod, 'demod': psk8_demod, 'bps': 3, 'order': 8, 'alpha': 0.012},
    '16QAM': {'mod': qam16_mod, 'demod': qam16_demod, 'bps': 4, 'order': 16, 'alpha': 0.006},
}


class SDRModem:
    """sdr_modem.py:17-342, modem part (mapping, hard demod, RRC shaping, IQ files)."""

    MODULATIONS = {
        'BPSK':   {'bps': 1, 'order': 2,   'alpha': 0.02,  'n_rot': 2, 'rot_step': np.pi},
        'QPSK':   {'bps': 2, 'order': 4,   'alpha': 0.015, 'n_rot': 4, 'rot_step': np.pi / 2},
        '8PSK':   {'bps': 3, 'order': 8,   'alpha': 0.01,  'n_rot': 8, 'rot_step': np.pi / 4},
        '16QAM':  {'bps': 4, 'order': 16,  'alpha': 0.008, 'n_rot': 4, 'rot_step': np.pi / 2},
        '64QAM':  {'bps': 6, 'order': 64,  'alpha': 0.005, 'n_rot': 4, 'rot_step': np.pi / 2},
        '256QAM': {'bps': 8, 'order': 256, 'alpha': 0.003, 'n_rot': 4, 'rot_step': np.pi / 2},
    }
    _QAM = {'16QAM': (2, 10), '64QAM': (3, 42), '256QAM': (4, 170)}

    def __init__(self, fc: float = 433e6, fs: float = 2e6, sps: int = 4, tx_gain: int = 47, rx_gain: int = 49,
                 device: int = 0):
        self.fc, self.fs, self.sps = fc, fs, sps
        self.tx_gain, self.rx_gain = tx_gain, rx_gain
        self.device = device
        self.rrc_taps = self._rrc_filter(sps)
        self.sync_bits = np.array([1, 0, 1, 0, 1, 0, 1, 0, 1, 1, 0, 0, 1, 1, 0, 0] * 10)
        self._sync_syms = None
        self._init_gray_tables()

    @property
    def sync_syms(self):
        if self._sync_syms is None:
            self._sync_syms = self._bpsk_mod(self.sync_bits)
        return self._sync_syms

    def _init_gray_tables(self):                     # :66-75
        self.gray2, self.gray3, self.gray4 = list(GRAY2), list(GRAY3), list(GRAY4)
        self.inv_gray2, self.inv_gray3, self.inv_gray4 = list(_INV[2]), list(_INV[3]), list(_INV[4])

    def _rrc_filter(self, sps: int, alpha: float = 0.35, ntaps: int = 101) -> np.ndarray:   # :77-91
        return _rrc_taps(sps, alpha, ntaps)

    def _upsample_filter(self, syms: np.ndarray) -> np.ndarray:                            # :93-97
        return _same_conv_up(syms, self.sps, self.rrc_taps, self.device)

    def _map(self, bits, mod):
        return map_bits(bits, self.MODULATIONS[mod]['bps'], _gray_table(mod), self.device)

    def _bpsk_mod(self, bits):
        return self._map(bits, 'BPSK')

    def _qpsk_mod(self, bits):
        return self._map(bits, 'QPSK')

    def _psk8_mod(self, bits):
        return self._map(bits, '8PSK')

    def _qam16_mod(self, bits):
        return self._map(bits, '16QAM')

    def _qam64_mod(self, bits):
        return self._map(bits, '64QAM')

    def _qam256_mod(self, bits):
        return self._map(bits, '256QAM')

    def _bpsk_demod(self, syms):
        return hard_demod(syms, GT0, 1, device=self.device).astype(int)

    def _qpsk_demod(self, syms):
        return hard_demod(syms, QPSK, 2, device=self.device).astype(int)

    def _psk8_demod(self, syms):
        return _loop_bits(hard_demod(syms, PSK8, 3, labels=_INV[3], nan_raises=True, device=self.device))

    def _qam_demod(self, syms, mod):
        k, s = self._QAM[mod]
        return _qam_demod(syms, k, np.sqrt(s), self.device)

    def _qam16_demod(self, syms):
        return self._qam_demod(syms, '16QAM')

    def _qam64_demod(self, syms):
        return self._qam_demod(syms, '64QAM')

    def _qam256_demod(self, syms):
        return self._qam_demod(syms, '256QAM')

    def modulate(self, bits: np.ndarray, modulation: str = 'QPSK') -> np.ndarray:          # :222-243
        if modulation not in self.MODULATIONS:
            raise ValueError(f"Unknown modulation: {modulation}")
        return self._map(bits, modulation)

    def demodulate(self, symbols: np.ndarray, modulation: str = 'QPSK') -> np.ndarray:     # :245-266
        f = {'BPSK': self._bpsk_demod, 'QPSK': self._qpsk_demod, '8PSK': self._psk8_demod,
             '16QAM': self._qam16_demod, '64QAM': self._qam64_demod, '256QAM': self._qam256_demod}
        if modulation not in f:
            raise ValueError(f"Unknown modulation: {modulation}")
        return f[modulation](symbols)

    def _save_iq(self, sig: np.ndarray, filename: str):                                    # :329-335
        save_iq(sig, filename, self.device)

    def _load_iq(self, filename: str) -> np.ndarray:                                       # :337-342
        return load_iq(filename, self.device)


# ---------------------------------------------------------------- natural family -------------
class Modulator:
    """modulators.py:50-199: natural-label mappers, argmin QAM demods, RRC
    pulse shaping (scipy upfirdn) and matched filtering."""

    def __init__(self, samples_per_symbol=8, bt=0.3, rrc_alpha=0.35, rrc_span=6, device=0):
        self.sps = int(samples_per_symbol)
        self.bt = float(bt)
        self.rrc_alpha = rrc_alpha
        self.rrc_span = rrc_span
        self.device = device
        self.rrc_filter = rrcosfilter(self.rrc_span, self.rrc_alpha, 1, self.sps)
        self.filter_delay = (len(self.rrc_filter) - 1) // 2
        self._tables = {}

    # ---- pulse shaping (:67-113)
    def apply_pulse_shaping(self, symbols):
        """upfirdn(h, syms, up=sps): (len-1)*sps + len(h) samples, complex128."""
        syms = np.array(symbols, dtype=np.complex64).ravel()
        if syms.size == 0:
            raise ValueError("x must be at least 1-D with at least 1 element")
        L = len(self.rrc_filter)
        return fir(syms, self.rrc_filter, up=self.sps, down=1, offset=0, n_out=(syms.size - 1) * self.sps + L,
                   device=self.device)

    def matched_filter(self, samples):
        """full convolution with h, then [2*delay::sps]."""
        x = np.asarray(samples)
        L = len(self.rrc_filter)
        n_full = x.size + L - 1
        start = 2 * self.filter_delay
        if start >= n_full:
            return np.array([], dtype=np.complex64)
        y = fir(x, self.rrc_filter, up=1, down=self.sps, offset=start, n_out=-(-(n_full - start) // self.sps),
                device=self.device)
        return y if np.iscomplexobj(x) else y.real.copy()

    # ---- tables: the reference expressions over every label
    def _table(self, name):
        t = self._tables.get(name)
        if t is None:
            if name == 'bpsk':
                t = (2 * np.arange(2) - 1).astype(np.complex64)                          # :119-120
            elif name == 'qpsk':
                b = np.array([[i >> 1, i & 1] for i in range(4)])
                t = ((1 - 2 * b[:, 0]) + 1j * (1 - 2 * b[:, 1])) / np.sqrt(2)           # :125-131
            elif name == '8psk':
                t = np.exp(1j * 2 * np.pi * np.arange(8) / 8)                             # :139-145
            else:
                t = self._qam_const(int(name[3:]))[0]                                     # :174-197
            self._tables[name] = t = np.ascontiguousarray(t)
        return t

    def _qam_const(self, M):                                                              # :157-163
        m = int(np.sqrt(M))
        axis = np.arange(-m + 1, m, 2)
        xv, yv = np.meshgrid(axis, axis)
        c = xv.flatten() + 1j * yv.flatten()
        c /= np.sqrt(np.mean(np.abs(c) ** 2))
        return c, axis

    def mod_bpsk(self, bits):
        return map_bits(bits, 1, self._table('bpsk'), self.device)

    def demod_bpsk(self, symbols):
        return hard_demod(symbols, GT0, 1, device=self.device).astype(int)

    def mod_qpsk(self, bits):
        return map_bits(bits, 2, self._table('qpsk'), self.device)

    def demod_qpsk(self, symbols):
        return hard_demod(symbols, QPSK, 2, device=self.device).astype(int)

    def mod_8psk(self, bits):
        return map_bits(bits, 3, self._table('8psk'), self.device)

    def demod_8psk(self, symbols):
        """astype(int) of a NaN angle is INT64_MIN on x86, and % 8 -> 0."""
        return _loop_bits(hard_demod(symbols, PSK8, 3, nan_raises=False, device=self.device))

    def _demod_qam_generic(self, symbols, M):
        k = int(np.log2(M))
        return _loop_bits(hard_demod(symbols, ARGMIN, k, cons=self._qam_const(M)[0], device=self.device))

    def mod_16qam(self, bits):
        return map_bits(bits, 4, self._table('qam16'), self.device)

    def demod_16qam(self, symbols):
        return self._demod_qam_generic(symbols, 16)

    def mod_64qam(self, bits):
        return map_bits(bits, 6, self._table('qam64'), self.device)

    def demod_64qam(self, symbols):
        return self._demod_qam_generic(symbols, 64)
