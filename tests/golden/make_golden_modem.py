#!/usr/bin/env python3
"""Generate the committed golden vectors of the modem front-end (SURVEY.md
§8(f) row 4): mappers, hard demodulators, RRC taps, pulse shaping, matched
filter and the IQ sample format.

TEST INFRASTRUCTURE ONLY.  Runs in the build container, where the read-only
reference checkout lives at /root/reference; it imports the reference's
``sdr_modem``, ``modulators`` and ``test_sdr_with_coding`` modules unmodified
(the last one after stubbing the stale ``DVB_RCS2_TurboCodec`` name it
imports and matplotlib, as make_golden.py does) and records inputs and
outputs as plain arrays in ``modem.npz``.  The IQ load vector uses the first
64 KiB of the reference's own capture ``tx.iq`` as input data.

Usage:  python tests/golden/make_golden_modem.py
"""
import os
import sys
import tempfile
import types
import warnings

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    sys.modules.setdefault("matplotlib", types.ModuleType("matplotlib"))
    mpl = sys.modules["matplotlib"]
    if not hasattr(mpl, "pyplot"):
        mpl.pyplot = types.ModuleType("matplotlib.pyplot")
        sys.modules["matplotlib.pyplot"] = mpl.pyplot
    shim = tempfile.mkdtemp(prefix="numba_shim_")
    os.makedirs(os.path.join(shim, "numba"))
    with open(os.path.join(shim, "numba", "__init__.py"), "w") as f:
        f.write("def njit(*a, **k):\n    if len(a) == 1 and callable(a[0]) and not k:\n        return a[0]\n"
                "    return lambda f: f\nint32 = float32 = float64 = int64 = None\n")
    sys.path.insert(0, shim)
    import dvb_rcs2_turbo as T
    T.DVB_RCS2_TurboCodec = None
    import sdr_modem as SM
    import modulators as MO
    import test_sdr_with_coding as H
    return SM, MO, H


def noisy(rng, const, n, sigma, dtype=np.complex64):
    tx = const[rng.integers(0, len(const), n)]
    return (tx + sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(dtype)


def main():
    SM, MO, H = _import()
    rng = np.random.default_rng(20251227)
    out = {}
    m = SM.SDRModem()   # construction only builds taps and tables (no radio)

    def err_of(fn, *a):
        try:
            fn(*a)
            return ""
        except Exception as e:   # noqa: BLE001 -- recorded, the tests compare type names
            return type(e).__name__

    # ---- SDRModem mappers / demods (sdr_modem.py:101-266) -------------------------------
    for mod, bps in (("BPSK", 1), ("QPSK", 2), ("8PSK", 3), ("16QAM", 4), ("64QAM", 6), ("256QAM", 8)):
        nb = 997 * bps + (1 if bps > 1 else 0)          # ragged: the mapper zero-pads
        bits = rng.integers(0, 2, nb)
        sy = m.modulate(bits, mod)
        out[f"sdr_bits_{mod}"] = bits
        out[f"sdr_mod_{mod}"] = sy
        all_bits = np.array([list(map(int, format(i, f"0{bps}b"))) for i in range(2 ** bps)]).ravel()
        const = m.modulate(all_bits, mod)
        rx = noisy(rng, const, 2000, 0.08)
        # edge symbols: exact points, decision boundaries, far outside, zeros, infinities
        edge = np.concatenate([const[:8].astype(np.complex64),
                               np.array([0, 1e-30, -1e-30j, 5 + 5j, -7 - 0.5j, np.inf, -np.inf + 1j,
                                         complex(0, np.inf), complex(1, -0.0), complex(-0.0, 0.0)], np.complex64)])
        if mod.endswith("QAM"):
            k, s = {"16QAM": (2, 10), "64QAM": (3, 42), "256QAM": (4, 170)}[mod]
            L = 1 << k
            mid = (2 * np.arange(L - 1) - (L - 2)) / np.sqrt(s)     # midpoints between levels: round-half-even ties
            edge = np.concatenate([edge, (mid + 1j * mid[::-1]).astype(np.complex64)])
        if mod == "8PSK":
            ang = (2 * np.arange(8) + 1) * np.pi / 8                 # sector boundaries
            edge = np.concatenate([edge, np.exp(1j * ang).astype(np.complex64), np.array([-1e-9 - 1j * 1e-12],
                                                                                         np.complex64)])
        rx = np.concatenate([edge, rx])
        out[f"sdr_rx_{mod}"] = rx
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            out[f"sdr_demod_{mod}"] = m.demodulate(rx, mod)
            rx128 = rx.astype(np.complex128)
            fin = np.isfinite(rx128)
            rx128[fin] *= 1 + 1e-9                             # off the float32 grid
            out[f"sdr_rx128_{mod}"] = rx128
            out[f"sdr_demod128_{mod}"] = m.demodulate(rx128, mod)
            out[f"sdr_nanerr_{mod}"] = np.array(err_of(m.demodulate, np.array([np.nan + 0j], np.complex64), mod))
            out[f"sdr_emptydemod_{mod}"] = m.demodulate(np.zeros(0, np.complex64), mod)
    out["sdr_unknown_err"] = np.array(err_of(m.modulate, np.zeros(4, int), "32APSK"))

    # ---- harness copies (test_sdr_with_coding.py:25-128, 228-240) -------------------------
    for mod in ("BPSK", "QPSK", "8PSK", "16QAM"):
        bps = H.MODULATIONS[mod]["bps"]
        bits = rng.integers(0, 2, 301 * bps + (1 if bps > 1 else 0))
        out[f"h_bits_{mod}"] = bits
        out[f"h_mod_{mod}"] = H.MODULATIONS[mod]["mod"](bits)
        rx = out[f"sdr_rx_{mod}"]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            out[f"h_demod_{mod}"] = H.MODULATIONS[mod]["demod"](rx)

    # ---- RRC taps and _upsample_filter ------------------------------------------------------
    for sps in (2, 4, 8):
        out[f"sdr_taps_{sps}"] = m._rrc_filter(sps)
    out["h_taps_4_025_65"] = H.rrc_taps(4, 0.25, 65)        # |t| == 1/(4 alpha) branch
    out["h_taps_8_05_33"] = H.rrc_taps(8, 0.5, 33)
    for n_sym, dt in ((500, np.complex64), (20, np.complex128), (7, np.complex64)):   # 7*4 < 101 taps: swapped
        syms = noisy(rng, out["sdr_mod_QPSK"], n_sym, 0.1, dt)
        out[f"sdr_upin_{n_sym}"] = syms
        out[f"sdr_upout_{n_sym}"] = m._upsample_filter(syms)
    out["h_upin"] = out["sdr_upin_500"]
    out["h_upout"] = H.upsample_filter(out["h_upin"], 8, out["sdr_taps_8"])

    # ---- IQ files ------------------------------------------------------------------------------
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "x.iq")
        sig = out["sdr_upout_500"]                           # complex128, as transmit() saves
        m._save_iq(sig, f)
        out["iq_sig128"] = sig
        out["iq_saved128"] = np.fromfile(f, np.int8)
        sig64 = (sig * 3.7).astype(np.complex64)
        m._save_iq(sig64, f)
        out["iq_sig64"] = sig64
        out["iq_saved64"] = np.fromfile(f, np.int8)
        tiny = np.array([1e-12 + 0j, -3e-11j, 0j], np.complex128)   # max|sig| below the 1e-10 guard
        m._save_iq(tiny, f)
        out["iq_sigtiny"] = tiny
        out["iq_savedtiny"] = np.fromfile(f, np.int8)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            weird = np.array([1 + 1j, np.nan + 0j, 0.5j], np.complex128)
            m._save_iq(weird, f)
            out["iq_signan"] = weird
            out["iq_savednan"] = np.fromfile(f, np.int8)
            weird = np.array([1 + 1j, np.inf + 0j, -0.5j], np.complex128)
            m._save_iq(weird, f)
            out["iq_siginf"] = weird
            out["iq_savedinf"] = np.fromfile(f, np.int8)
        raw = np.fromfile(os.path.join(REF, "tx.iq"), np.uint8, count=65536)
        f2 = os.path.join(d, "r.iq")
        np.concatenate([raw, np.arange(256, dtype=np.uint8)]).tofile(f2)
        out["iq_raw"] = np.fromfile(f2, np.uint8)
        out["iq_loaded"] = m._load_iq(f2)
        h = H.load_iq(f2)
        out["iq_loaded_h"] = h
        raw[:3].tofile(f2)
        out["iq_odd_err"] = np.array(err_of(m._load_iq, f2))
        out["iq_empty_err"] = np.array(err_of(m._save_iq, np.zeros(0, np.complex128), f2))

    # ---- Modulator (modulators.py) ----------------------------------------------------------
    out["mo_rrc_6_035_1_8"] = MO.rrcosfilter(6, 0.35, 1, 8)
    out["mo_rrc_4_025_1_8"] = MO.rrcosfilter(4, 0.25, 1, 8)   # |t| == Ts/(4 alpha)
    out["mo_rrc_3_0_1_4"] = MO.rrcosfilter(3, 0.0, 1, 4)      # alpha = 0
    out["mo_rrc_5_05_2_4"] = MO.rrcosfilter(5, 0.5, 2, 4)     # Ts = 2
    mo = MO.Modulator()
    for name, bps in (("bpsk", 1), ("qpsk", 2), ("8psk", 3), ("16qam", 4), ("64qam", 6)):
        bits = rng.integers(0, 2, 499 * bps + (1 if bps > 1 else 0))
        sy = getattr(mo, f"mod_{name}")(bits)
        out[f"mo_bits_{name}"] = bits
        out[f"mo_mod_{name}"] = sy
        all_bits = np.array([list(map(int, format(i, f"0{bps}b"))) for i in range(2 ** bps)]).ravel()
        const = getattr(mo, f"mod_{name}")(all_bits)
        rx = noisy(rng, const, 1500, 0.1)
        edge = np.array([0, 5 + 5j, -3 - 0.1j, np.inf, complex(0, -np.inf), complex(-0.0, 0.0)], np.complex64)
        if name == "8psk":
            edge = np.concatenate([edge, np.exp(1j * (2 * np.arange(8) + 1) * np.pi / 8).astype(np.complex64)])
        if name in ("16qam", "64qam"):
            edge = np.concatenate([edge, const[:6].astype(np.complex64),
                                   ((const[0] + const[1]) / 2).astype(np.complex64)[None]])   # tie: first index
        rx = np.concatenate([edge, rx])
        out[f"mo_rx_{name}"] = rx
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            out[f"mo_demod_{name}"] = getattr(mo, f"demod_{name}")(rx)
            rx128 = rx.astype(np.complex128)
            out[f"mo_demod128_{name}"] = getattr(mo, f"demod_{name}")(rx128)
            nanrx = np.array([np.nan + 0j, 1 + 1j], np.complex64)
            out[f"mo_nanrx_{name}"] = nanrx
            out[f"mo_nandemod_{name}"] = getattr(mo, f"demod_{name}")(nanrx)
    syms = out["mo_mod_qpsk"][:300]
    out["mo_shape_in"] = syms
    shaped = mo.apply_pulse_shaping(syms)
    out["mo_shaped"] = shaped
    out["mo_mf_in"] = shaped
    out["mo_mf_out"] = mo.matched_filter(shaped)
    mf64 = shaped.astype(np.complex64)
    out["mo_mf64_in"] = mf64
    out["mo_mf64_out"] = mo.matched_filter(mf64)
    out["mo_mf_short_out"] = mo.matched_filter(shaped[:10])     # shorter than the 2*delay start
    out["mo_mf_real_in"] = shaped.real.copy()
    out["mo_mf_real_out"] = mo.matched_filter(shaped.real.copy())
    np.savez_compressed(os.path.join(OUT, "modem.npz"), **out)
    print("wrote", os.path.join(OUT, "modem.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
