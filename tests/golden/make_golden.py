#!/usr/bin/env python3
"""Generate the committed golden vectors for the turbo-decode hot path.

TEST INFRASTRUCTURE ONLY.  This script runs in the survey/build container,
where the read-only reference checkout lives at /root/reference.  It imports
the reference's ``dvb_rcs2_turbo`` module unmodified, with a no-op ``numba``
stand-in (``njit`` = identity) so the numba kernels run as plain
CPython + numpy.  SURVEY.md §8(c) records that this shim is bit-identical to
the author's cached numba machine code for ``bcjr_max_log_map``.

The reference never travels to the GPU box: only the ``*.npz`` files written
here (inputs and expected outputs, no code) do.

Which inverse interleaver a vector used is recorded per file
(``inv_perm`` key), because ``np.argsort(perm)`` of the reference
(dvb_rcs2_turbo.py:325) breaks ties differently per numpy SIMD path
(SURVEY.md fact 4).  ``inv_stable`` = ``np.argsort(perm, kind='stable')`` is the
build's canonical pin; ``inv_default`` is what this container's numpy
(2.2.6, AVX-512) returns for the reference's unstable argsort.

Usage:  python tests/golden/make_golden.py   (takes a few minutes)
"""
import os
import sys
import tempfile
import time

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

N_ALL = [48, 64, 212, 220, 424, 752, 848]


def _import_reference():
    shim = tempfile.mkdtemp(prefix="numba_shim_")
    os.makedirs(os.path.join(shim, "numba"))
    with open(os.path.join(shim, "numba", "__init__.py"), "w") as f:
        f.write(
            "def njit(*a, **k):\n"
            "    if len(a) == 1 and callable(a[0]) and not k:\n"
            "        return a[0]\n"
            "    return lambda f: f\n"
            "int32 = float32 = float64 = int64 = None\n"
        )
    sys.path[:0] = [shim, REF]
    sys.dont_write_bytecode = True
    import dvb_rcs2_turbo as T  # noqa: E402
    return T


def make_codec(T, n, rate, iterations=8):
    """Construct without the (slow, pure-Python) JIT warm-up decode."""
    orig = T.DVBRCS2_Turbo.decode
    T.DVBRCS2_Turbo.decode = lambda self, llr: None
    try:
        c = T.DVBRCS2_Turbo(n, rate, iterations)
    finally:
        T.DVBRCS2_Turbo.decode = orig
    return c


def gen_tables(T):
    c = make_codec(T, 48, "1/3")
    out = dict(
        next_state=c.next_state, out_W=c.out_W, out_Y=c.out_Y,
        prev_state=c.prev_state, prev_input=c.prev_input, G=c.G_matrix,
        N_all=np.array(N_ALL, np.int32),
        interleaver_params=np.array([T.INTERLEAVER_PARAMS[n] for n in N_ALL], np.int32),
    )
    for n in N_ALL:
        cc = make_codec(T, n, "1/3")
        out[f"perm_{n}"] = cc.perm
        out[f"inv_default_{n}"] = cc.inv_perm
        out[f"inv_stable_{n}"] = np.argsort(cc.perm, kind="stable").astype(np.int32)
        for rate in ("1/3", "1/2", "2/3", "3/4"):
            out[f"n_coded_{n}_{rate.replace('/', '_')}"] = np.int64(make_codec(T, n, rate).n_coded)
    # G^N and the circular-state solution for every Z_N (encoder, :404-429)
    for n in N_ALL:
        gp = T.mat_pow_gf2(c.G_matrix, n)
        out[f"gpow_{n}"] = gp
        out[f"circ_{n}"] = np.array([T.solve_circular_state_gf2(gp, z) for z in range(16)], np.int32)
    np.savez_compressed(os.path.join(OUT, "tables.npz"), **out)


def gen_encode(T):
    rng = np.random.default_rng(20251226)
    out = {}
    for n, rates in ((48, ("1/3", "1/2", "2/3", "3/4")), (212, ("1/3", "1/2")), (752, ("1/3", "1/2"))):
        for rate in rates:
            c = make_codec(T, n, rate)
            bits = rng.integers(0, 2, (6, c.k_info)).astype(np.int32)
            coded = np.stack([c.encode(b) for b in bits])
            key = f"{n}_{rate.replace('/', '_')}"
            out[f"bits_{key}"] = bits
            out[f"coded_{key}"] = coded
    np.savez_compressed(os.path.join(OUT, "encode.npz"), **out)


def gen_siso(T):
    """Per-SISO known answers: bcjr_max_log_map (dvb_rcs2_turbo.py:116-281)."""
    rng = np.random.default_rng(7)
    c = make_codec(T, 48, "1/3")
    tabs = (c.next_state, c.out_W, c.out_Y, c.prev_state, c.prev_input)
    out = {}
    for n, count in ((48, 10), (212, 6), (752, 4)):
        cases = []
        for i in range(count):
            sc = [0.5, 2.0, 8.0, 30.0][i % 4]
            la_sc = [0.0, 5.0, 20.0, 50.0][(i // 2) % 4]
            Lc = (rng.standard_normal((4, n)) * sc).astype(np.float32)
            La = rng.standard_normal((2, n)) * la_sc
            if i == 1:   # all-zero input: ties everywhere
                Lc[:] = 0
                La[:] = 0
            if i == 2:   # saturating extrinsic (clip at +-300) and big parities
                Lc *= 200
                La *= 20
            sf = 0.7 if i % 3 else 1.0
            cases.append((Lc, La, sf))
        LcA = np.stack([x[0][0] for x in cases]); LcB = np.stack([x[0][1] for x in cases])
        LcW = np.stack([x[0][2] for x in cases]); LcY = np.stack([x[0][3] for x in cases])
        LaA = np.stack([x[1][0] for x in cases]); LaB = np.stack([x[1][1] for x in cases])
        sf = np.array([x[2] for x in cases])
        LeA = np.zeros_like(LaA); LeB = np.zeros_like(LaB)
        for j in range(count):
            LeA[j], LeB[j] = T.bcjr_max_log_map(LcA[j], LcB[j], LcW[j], LcY[j], LaA[j], LaB[j],
                                                 *tabs, n, float(sf[j]))
        out.update({f"LcA_{n}": LcA, f"LcB_{n}": LcB, f"LcW_{n}": LcW, f"LcY_{n}": LcY,
                    f"LaA_{n}": LaA, f"LaB_{n}": LaB, f"sf_{n}": sf,
                    f"LeA_{n}": LeA, f"LeB_{n}": LeB})
    np.savez_compressed(os.path.join(OUT, "siso.npz"), **out)


def gen_siso_f64(T):
    """bcjr_max_log_map with FLOAT64 channel LLRs: numba
    specialises the same source for f64 Lc, so in_A = Lc_A + La_A and the parity
    terms are formed from the unrounded values (:135-160) and the extrinsic
    subtracts the f64 sum (:267-268).  All-f64 arithmetic is the same under numba
    and CPython + numpy, so the shim pins it.  Also: a mixed call (f64 A / W, f32
    B / Y: numba widens the f32 ones, numpy does too in every sum that has an f64
    operand) and integer channel LLRs (int64 + f64 -> f64 in both).  Rows per N:
    random scales, values f32 cannot hold (1e-310 denormals, 1e39, 0.1 + 1e-12),
    NaN / +-inf, sf 0.7 and 1.0."""
    rng = np.random.default_rng(64)
    c = make_codec(T, 48, "1/3")
    tabs = (c.next_state, c.out_W, c.out_Y, c.prev_state, c.prev_input)
    out = {}
    for n, count in ((48, 12), (212, 8), (752, 6)):
        rows = []
        for i in range(count):
            sc = [0.3, 2.0, 9.0, 40.0][i % 4]
            la_sc = [0.0, 4.0, 25.0, 80.0][(i // 2) % 4]
            Lc = rng.standard_normal((4, n)) * sc
            La = rng.standard_normal((2, n)) * la_sc
            kind = i % 6
            if kind == 1:   # just off the f32 grid: every value differs from its f32 rounding
                Lc = Lc + 1e-9 * rng.standard_normal((4, n))
            elif kind == 2:   # f64-only magnitudes: denormals and values beyond f32's range
                pos = rng.integers(0, n, max(3, n // 8))
                Lc[2, pos] = 1e-310 * rng.standard_normal(len(pos))
                Lc[3, pos[::2]] = 3e39 * np.sign(rng.standard_normal(len(pos[::2])))
                Lc[0, pos[1::3]] = -4e-320
            elif kind == 3:   # non-finite channel values
                pos = rng.integers(0, n, max(2, n // 16))
                Lc[rng.integers(0, 4), pos] = np.nan
                Lc[rng.integers(0, 4), pos[::2]] = np.inf
                Lc[1, pos[1::2]] = -np.inf
            elif kind == 4:   # saturating extrinsics (+-300 clip)
                Lc *= 150.0
                La *= 10.0
            sf = 0.7 if i % 3 else 1.0
            a, b = T.bcjr_max_log_map(Lc[0], Lc[1], Lc[2], Lc[3], La[0], La[1], *tabs, n, sf)
            rows.append((Lc, La, sf, a, b))
        out[f"Lc_{n}"] = np.stack([r[0] for r in rows])          # [count, 4, n] float64
        out[f"La_{n}"] = np.stack([r[1] for r in rows])          # [count, 2, n] float64
        out[f"sf_{n}"] = np.array([r[2] for r in rows])
        out[f"LeA_{n}"] = np.stack([r[3] for r in rows])
        out[f"LeB_{n}"] = np.stack([r[4] for r in rows])
        print(f"  siso_f64 N={n}", flush=True)
    # a mixed-dtype call and an integer-Lc call per N (N = 48, 212)
    for n in (48, 212):
        Lc = rng.standard_normal((4, n)) * 5.0 + 1e-7
        La = rng.standard_normal((2, n)) * 12.0
        A, B, W, Y = Lc[0], Lc[1].astype(np.float32), Lc[2], Lc[3].astype(np.float32)
        a, b = T.bcjr_max_log_map(A, B, W, Y, La[0], La[1], *tabs, n, 0.7)
        out.update({f"mix_A_{n}": A, f"mix_B_{n}": B, f"mix_W_{n}": W, f"mix_Y_{n}": Y, f"mix_La_{n}": La,
                    f"mix_LeA_{n}": a, f"mix_LeB_{n}": b})
        I = rng.integers(-40, 41, (4, n)).astype(np.int64)
        a, b = T.bcjr_max_log_map(I[0], I[1], I[2], I[3], La[0], La[1], *tabs, n, 1.0)
        out.update({f"int_Lc_{n}": I, f"int_La_{n}": La, f"int_LeA_{n}": a, f"int_LeB_{n}": b})
    np.savez_compressed(os.path.join(OUT, "siso_f64.npz"), **out)


class _Capture:
    """Wrap T.bcjr_max_log_map (resolved as a module global at call time by
    DVBRCS2_Turbo.decode, dvb_rcs2_turbo.py:499/515) to record SISO I/O."""

    def __init__(self, T):
        self.T = T
        self.fn = T.bcjr_max_log_map
        self.calls = []

    def __enter__(self):
        def wrapped(*a):
            r = self.fn(*a)
            self.calls.append((a[0], a[4], a[5], r[0], r[1]))
            return r
        self.T.bcjr_max_log_map = wrapped
        return self

    def __exit__(self, *exc):
        self.T.bcjr_max_log_map = self.fn


def _decode_capture(T, c, llr):
    with _Capture(T) as cap:
        bits = c.decode(llr)
    # Final decision (dvb_rcs2_turbo.py:529-530): Lc + La + Le1, La = Le2[inv_perm]
    LcA1, _, _, Le1A, Le1B = cap.calls[-2]
    _, _, _, Le2A, Le2B = cap.calls[-1]
    LcA = LcA1
    llr32 = np.array(llr, dtype=np.float32)
    LcB = np.zeros(c.N, np.float32)
    # recover Lc_B the same way decode() depunctures it (systematic B is the 2nd value of each couple)
    idx = 0
    per = c.punct["period"]
    for i in range(c.N):
        p = i % per
        idx += 1
        LcB[i] = llr32[idx]; idx += 1
        idx += c.punct["W1"][p] + c.punct["Y1"][p] + c.punct["W2"][p] + c.punct["Y2"][p]
    LaA = Le2A[c.inv_perm]; LaB = Le2B[c.inv_perm]
    LfA = LcA + LaA + Le1A
    LfB = LcB + LaB + Le1B
    lfinal = np.zeros(2 * c.N)
    lfinal[0::2] = LfA; lfinal[1::2] = LfB
    assert np.array_equal(bits[0::2], (LfA < 0).astype(np.int32))
    return bits, lfinal


def _qpsk_llrs(rng, coded, ebn0_db, rate):
    """AWGN + QPSK LLRs, decoder sign (LLR>0 => bit 0), SURVEY.md §8(d)."""
    a = coded[0::2]; b = coded[1::2]
    sym = ((1 - 2.0 * a) + 1j * (1 - 2.0 * b)) / np.sqrt(2)
    n0 = 1.0 / (rate * 2 * 10 ** (ebn0_db / 10.0))
    sig = np.sqrt(n0 / 2)
    y = sym + sig * (rng.standard_normal(sym.shape) + 1j * rng.standard_normal(sym.shape))
    llr = np.zeros(coded.shape[0], np.float32)
    llr[0::2] = 2 * np.sqrt(2) * y.real / n0
    llr[1::2] = 2 * np.sqrt(2) * y.imag / n0
    return llr


def gen_decode(T):
    """Full-decode known answers: DVBRCS2_Turbo.decode (dvb_rcs2_turbo.py:464-537)."""
    rng = np.random.default_rng(99)
    out = {}
    plan = [(48, "1/3", 6), (48, "1/2", 4), (48, "2/3", 2), (212, "1/3", 4), (212, "1/2", 3),
            (752, "1/3", 3), (752, "1/2", 2)]
    for n, rate, count in plan:
        Rn = {"1/3": 1 / 3, "1/2": 1 / 2, "2/3": 2 / 3, "3/4": 3 / 4}[rate]
        for variant in ("stable", "default"):
            if variant == "default" and rate != "1/3":
                continue
            c = make_codec(T, n, rate)
            if variant == "stable":
                c.inv_perm = np.argsort(c.perm, kind="stable").astype(np.int32)
            key = f"{n}_{rate.replace('/', '_')}_{variant}"
            bits_in, llrs, bits_out, lfin, ebn0 = [], [], [], [], []
            for i in range(count):
                info = rng.integers(0, 2, c.k_info).astype(np.int32)
                coded = c.encode(info)
                e = [0.0, 2.0, 4.0, 99.0][i % 4]
                if e == 99.0:
                    llr = (1 - 2.0 * coded).astype(np.float32) * 20.0
                else:
                    llr = _qpsk_llrs(rng, coded, e, Rn)
                if len(llr) < c.n_coded:  # rate-2/3 quirk: encode() length != n_coded
                    llr = np.pad(llr, (0, c.n_coded - len(llr)))
                t = time.time()
                b, lf = _decode_capture(T, c, llr)
                print(f"  decode {key} #{i} ebn0={e} errs={int((b != info).sum())} "
                      f"({time.time() - t:.1f}s)", flush=True)
                bits_in.append(info); llrs.append(llr); bits_out.append(b); lfin.append(lf); ebn0.append(e)
            out[f"info_{key}"] = np.stack(bits_in)
            out[f"llr_{key}"] = np.stack(llrs)
            out[f"bits_{key}"] = np.stack(bits_out)
            out[f"lfinal_{key}"] = np.stack(lfin)
            out[f"ebn0_{key}"] = np.array(ebn0)
            out[f"inv_{key}"] = c.inv_perm
    # The survey's behavioural KATs: noise-free +-20 LLRs,
    # info bits from default_rng(1), container-default inv_perm.
    for n in (48, 212, 752):
        c = make_codec(T, n, "1/3")
        info = np.random.default_rng(1).integers(0, 2, c.k_info)
        coded = c.encode(info)
        b = c.decode((1 - 2 * coded) * 20.0)
        out[f"kat_info_{n}"] = info.astype(np.int32)
        out[f"kat_bits_{n}"] = b
        out[f"kat_inv_{n}"] = c.inv_perm
        print(f"  KAT N={n}: {int((b != info).sum())} errors", flush=True)
    np.savez_compressed(os.path.join(OUT, "decode.npz"), **out)


def gen_nonfinite(T):
    """Non-finite inputs through the reference: SISO calls and
    full decodes whose LLRs / a-priori values hold NaN, +inf, -inf (scattered,
    whole rows, mixed), and the harness chain compute_llr -> decode with NaN and
    inf symbols (test_sdr_with_coding.py:213-225: a NaN symbol gives NaN LLRs).
    The reference's strict `>` recursions (:174-176, :247-248) drop NaN
    candidates and its `if` clip (:276-279) passes NaN through; these vectors
    pin what that does end to end."""
    rng = np.random.default_rng(2024)
    c = make_codec(T, 48, "1/3")
    tabs = (c.next_state, c.out_W, c.out_Y, c.prev_state, c.prev_input)
    out = {}
    kinds = ("nan", "pinf", "ninf", "mixed", "row_nan", "la_nan", "la_inf", "inf_both")
    for n in (48, 212, 752):
        LcA, LcB, LcW, LcY, LaA, LaB, LeA, LeB = ([] for _ in range(8))
        for kind in kinds:
            Lc = (rng.standard_normal((4, n)) * 3.0).astype(np.float32)
            La = rng.standard_normal((2, n)) * 6.0
            pos = rng.integers(0, n, max(2, n // 16))
            if kind == "nan":
                Lc[rng.integers(0, 4), pos] = np.nan
            elif kind == "pinf":
                Lc[rng.integers(0, 4), pos] = np.inf
            elif kind == "ninf":
                Lc[rng.integers(0, 4), pos] = -np.inf
            elif kind == "mixed":
                Lc[0, pos[0::3]] = np.nan
                Lc[2, pos[1::3]] = np.inf
                Lc[3, pos[2::3]] = -np.inf
            elif kind == "row_nan":
                Lc[1, :] = np.nan
            elif kind == "la_nan":
                La[0, pos] = np.nan
            elif kind == "la_inf":
                La[1, pos] = np.inf
                La[0, pos[::2]] = -np.inf
            elif kind == "inf_both":
                Lc[0, pos] = np.inf
                Lc[1, pos] = -np.inf
            a, b = T.bcjr_max_log_map(Lc[0], Lc[1], Lc[2], Lc[3], La[0], La[1], *tabs, n, 0.7)
            for lst, v in zip((LcA, LcB, LcW, LcY, LaA, LaB, LeA, LeB), (*Lc, *La, a, b)):
                lst.append(v)
        out.update({f"siso_{k}_{n}": np.stack(v) for k, v in
                    zip(("LcA", "LcB", "LcW", "LcY", "LaA", "LaB", "LeA", "LeB"),
                        (LcA, LcB, LcW, LcY, LaA, LaB, LeA, LeB))})
    out["siso_kinds"] = np.array(kinds)
    # full decodes (stable inverse interleaver, as the decode.npz 'stable' vectors)
    for n, rate in ((48, "1/3"), (212, "1/3"), (752, "1/2")):
        cc = make_codec(T, n, rate)
        cc.inv_perm = np.argsort(cc.perm, kind="stable").astype(np.int32)
        key = f"{n}_{rate.replace('/', '_')}"
        llrs, bits, lfs = [], [], []
        for kind in ("nan", "pinf", "ninf", "mixed", "row_nan"):
            info = rng.integers(0, 2, cc.k_info)
            llr = ((1 - 2.0 * cc.encode(info)) * 2.0 + rng.standard_normal(cc.n_coded) * 1.2).astype(np.float32)
            pos = rng.integers(0, cc.n_coded, max(3, cc.n_coded // 40))
            if kind == "nan":
                llr[pos] = np.nan
            elif kind == "pinf":
                llr[pos] = np.inf
            elif kind == "ninf":
                llr[pos] = -np.inf
            elif kind == "mixed":
                llr[pos[0::3]] = np.nan
                llr[pos[1::3]] = np.inf
                llr[pos[2::3]] = -np.inf
            else:
                llr[:] = np.nan
            t = time.time()
            b, lf = _decode_capture(T, cc, llr)
            print(f"  nonfinite decode {key} {kind} ({time.time() - t:.1f}s)", flush=True)
            llrs.append(llr); bits.append(b); lfs.append(lf)
        out[f"dec_llr_{key}"] = np.stack(llrs)
        out[f"dec_bits_{key}"] = np.stack(bits)
        out[f"dec_lfinal_{key}"] = np.stack(lfs)
        out[f"dec_inv_{key}"] = cc.inv_perm
    # the harness chain: 16QAM symbols with NaN / inf entries -> compute_llr
    # (test_sdr_with_coding.py:200-225) -> the decoder's sign -> decode (N=212, r=1/3)
    import types
    T.DVB_RCS2_TurboCodec = None
    sys.modules.setdefault("matplotlib", types.ModuleType("matplotlib"))
    mpl = sys.modules["matplotlib"]
    if not hasattr(mpl, "pyplot"):
        mpl.pyplot = types.ModuleType("matplotlib.pyplot")
        sys.modules["matplotlib.pyplot"] = mpl.pyplot
    import test_sdr_with_coding as H
    cc = make_codec(T, 212, "1/3")
    cc.inv_perm = np.argsort(cc.perm, kind="stable").astype(np.int32)
    info = rng.integers(0, 2, cc.k_info)
    coded = cc.encode(info)
    syms = H.MODULATIONS["16QAM"]["mod"](coded).astype(np.complex64)
    syms = (syms + 0.25 * (rng.standard_normal(syms.shape) + 1j * rng.standard_normal(syms.shape))).astype(np.complex64)
    syms[[3, 77, 200]] = np.complex64(complex(np.nan, 0.5))
    syms[[10, 11]] = np.complex64(complex(np.inf, -1.0))
    syms[150] = np.complex64(complex(np.nan, np.nan))
    llr = -H.compute_llr(syms, "16QAM", np.float64(0.1))
    b, lf = _decode_capture(T, cc, llr)
    out.update(chain_syms=syms, chain_llr=llr, chain_bits=b, chain_lfinal=lf, chain_inv=cc.inv_perm,
               chain_noise_var=np.float64(0.1))
    np.savez_compressed(os.path.join(OUT, "nonfinite.npz"), **out)


def gen_demap():
    """compute_llr (test_sdr_with_coding.py:200-225) and the Gray mappers
    (:25-100; sdr_modem.py:101-220).  test_sdr_with_coding imports a stale
    name from dvb_rcs2_turbo, which is stubbed before import."""
    import types
    import dvb_rcs2_turbo as T
    T.DVB_RCS2_TurboCodec = None
    sys.modules.setdefault("matplotlib", types.ModuleType("matplotlib"))
    mpl = sys.modules["matplotlib"]
    if not hasattr(mpl, "pyplot"):
        mpl.pyplot = types.ModuleType("matplotlib.pyplot")
        sys.modules["matplotlib.pyplot"] = mpl.pyplot
    import test_sdr_with_coding as H
    import sdr_modem as SM
    rng = np.random.default_rng(5)
    out = {}
    for mod in ("BPSK", "QPSK", "8PSK", "16QAM"):
        bps = H.MODULATIONS[mod]["bps"]
        order = H.MODULATIONS[mod]["order"]
        all_bits = np.array([list(map(int, format(i, f"0{bps}b"))) for i in range(order)])
        const = H.MODULATIONS[mod]["mod"](all_bits.flatten()).reshape(-1)
        out[f"const_{mod}"] = const
        nsym = 300
        tx = const[rng.integers(0, order, nsym)]
        syms = (tx + 0.3 * (rng.standard_normal(nsym) + 1j * rng.standard_normal(nsym))).astype(np.complex64)
        syms[:4] = const[:4] if order >= 4 else syms[:4]  # exact constellation hits -> ties / zero distances
        out[f"syms_{mod}"] = syms
        out[f"llr_f64nv_{mod}"] = H.compute_llr(syms, mod, np.float64(0.137))   # call-site dtype (:464-471)
        out[f"llr_f64nvsmall_{mod}"] = H.compute_llr(syms, mod, np.float64(0.001))  # floor at 0.005
        out[f"llr_pyfloat_{mod}"] = H.compute_llr(syms, mod, 0.02)                # python float: f32 division
        out[f"llr_c128_{mod}"] = H.compute_llr(syms.astype(np.complex128) * (1 + 1e-9), mod, np.float64(0.2))
    m = SM.SDRModem.__new__(SM.SDRModem)
    m._init_gray_tables()
    for mod, bps in (("8PSK", 3), ("16QAM", 4), ("64QAM", 6), ("256QAM", 8)):
        all_bits = np.array([list(map(int, format(i, f"0{bps}b"))) for i in range(2 ** bps)])
        out[f"sdrconst_{mod}"] = m.modulate(all_bits.flatten(), mod).reshape(-1)
    np.savez_compressed(os.path.join(OUT, "demap.npz"), **out)


def main():
    T = _import_reference()
    t0 = time.time()
    if "--only" in sys.argv:   # one generator, e.g. --only nonfinite
        globals()["gen_" + sys.argv[sys.argv.index("--only") + 1]](T)
        return
    gen_tables(T); print("tables", time.time() - t0, flush=True)
    gen_encode(T); print("encode", time.time() - t0, flush=True)
    gen_siso(T); print("siso", time.time() - t0, flush=True)
    gen_demap(); print("demap", time.time() - t0, flush=True)
    gen_decode(T); print("decode", time.time() - t0, flush=True)
    gen_nonfinite(T); print("nonfinite", time.time() - t0, flush=True)


if __name__ == "__main__":
    main()
