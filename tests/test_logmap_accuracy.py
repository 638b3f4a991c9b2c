"""Accuracy of the build-defined log-MAP against log-MAP in exact f64 arithmetic
(the reference has no log-MAP source, so
there is no external parity to pin -- these tests bound the distance to the
mathematical definition instead).

The exact reference is the C oracle's algo=2 (oracle/tdec_oracle.c
siso_exact: the SISO of dvb_rcs2_turbo.py:116-281 with every max replaced by
max(a,b) + log1p(exp(-|a-b|)) in f64, branch metrics unrounded), pinned here to
an independent numpy restatement (np.logaddexp).

Stated tolerances:
* one SISO: |Le - Le_exact| <= 1e-5 + 4 ulp_f32(M), M = the block's largest
  |Lc + La| -- the recursions are f32 (as the reference's max-log), so no f32
  log-MAP can resolve 1e-5 once the metrics exceed ~64;
* a full 8-iteration decode (configs[3]: 8PSK, N=752 couples, r=1/2):
  |L_final - L_exact| <= 2e-3 * max(1, |L_exact|) -- the turbo loop feeds each
  SISO's rounding into the next 15; measured 3e-5..4e-4 relative at 1-3 dB --
  and identical hard bits wherever |L_exact| > 1e-2.
The unpinned comparison (GPU against the oracle with correctly rounded exp2 /
log2 instead of the device's tables) is here too: it differs only by the
hardware primitives' 1-ulp deviations."""
import numpy as np
import pytest

from oracle import oracle as O
from modulations_amd import dvb_rcs2_turbo as M
from modulations_amd import demap as D
from modulations_amd import tables as T

TAB, _ = O.trellis()


def _exact_np(Lc, La, sf):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_oracle_golden import _logmap_f64_exact
    return _logmap_f64_exact(Lc, La, sf, TAB)


def _siso_tol(Lc, La):
    big = max(np.max(np.abs(Lc[0] + La[0])), np.max(np.abs(Lc[1] + La[1])), 1.0)
    return 1e-5 + 4 * np.spacing(np.float32(big)).astype(np.float64)


def _8psk_llrs(codec, B, ebn0, seed):
    """configs[3]'s chain on the host: Gray 8PSK over AWGN, the decoder-sign soft
    demap (compute_llr, test_sdr_with_coding.py:200-225), truncated to n_coded."""
    rng = np.random.default_rng(seed)
    cons = D.constellation("8PSK")
    info = rng.integers(0, 2, (B, codec.k_info))
    rate = 2 * codec.N / codec.n_coded
    n0 = 1.0 / (rate * 3 * 10 ** (ebn0 / 10))
    out = []
    for b in info:
        bits = np.concatenate([codec.encode(b), [0]])           # 3008 bits + 1 pad -> 1003 symbols
        lab = bits.reshape(-1, 3) @ np.array([4, 2, 1])
        s = cons[lab] + np.sqrt(n0 / 2) * (rng.standard_normal(lab.size) + 1j * rng.standard_normal(lab.size))
        _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
        out.append(-O.demap(s.astype(np.complex64), cons, 3, nve, div_f32=div32)[:codec.n_coded])
    return np.stack(out).astype(np.float32)


def _oracle_decode(codec, llr, algo):
    return O.decode_batch(llr, codec.N, codec.punct["period"], T.puncture_matrix(codec.punct), codec.iterations,
                          codec.perm, codec.inv_perm, TAB, algo=algo, want_lfinal=True, nthreads=8)


def _check_decode(bits, lf, ebits, elf):
    assert np.all(np.abs(lf - elf) <= 2e-3 * np.maximum(1.0, np.abs(elf)))
    sure = np.abs(elf) > 1e-2
    assert np.array_equal(bits[sure], ebits[sure])


@pytest.mark.parametrize("n,sc,lsc", [(48, 1, 3), (212, 2, 8), (100, 8, 40)])
def test_exact_oracle_equals_numpy_logaddexp(n, sc, lsc):
    rng = np.random.default_rng(n)
    Lc = (rng.standard_normal((4, n)) * sc).astype(np.float32)
    La = rng.standard_normal((2, n)) * lsc
    A, B = O.siso(*Lc, *La, TAB, 0.7, algo=2)
    RA, RB = _exact_np(Lc, La, 0.7)
    assert np.max(np.abs(A - RA)) < 1e-9 and np.max(np.abs(B - RB)) < 1e-9


@pytest.mark.parametrize("n,sc,lsc", [(48, 1, 3), (212, 2, 8), (752, 3, 10), (212, 6, 20), (100, 8, 40)])
def test_cpu_logmap_siso_vs_exact(n, sc, lsc):
    rng = np.random.default_rng(7 * n + sc)
    Lc = (rng.standard_normal((4, n)) * sc).astype(np.float32)
    La = rng.standard_normal((2, n)) * lsc
    A, B = O.siso(*Lc, *La, TAB, 0.7, algo=1)
    RA, RB = O.siso(*Lc, *La, TAB, 0.7, algo=2)
    tol = _siso_tol(Lc, La)
    assert max(np.max(np.abs(A - RA)), np.max(np.abs(B - RB))) <= tol


@pytest.mark.parametrize("ebn0", [1.0, 3.0])
def test_cpu_logmap_full_decode_vs_exact(ebn0):
    c = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    llr = _8psk_llrs(c, 3, ebn0, int(ebn0 * 10))
    bits, lf = _oracle_decode(c, llr, 1)
    eb, elf = _oracle_decode(c, llr, 2)
    _check_decode(bits, lf, eb, elf)


# ---- GPU (no trans_tables fixture: the oracle keeps the correctly rounded primitives) --

def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.gpu
@pytest.mark.parametrize("ebn0", [1.0, 2.0, 3.0])
def test_gpu_logmap_full_decode_vs_exact(ebn0):
    """configs[3] inputs through the GPU's log-MAP decoder against exact f64 log-MAP."""
    _gpu()
    c = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    llr = _8psk_llrs(c, 8, ebn0, 100 + int(ebn0 * 10))
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    eb, elf = _oracle_decode(c, llr, 2)
    _check_decode(bits, lf, eb, elf)


@pytest.mark.gpu
@pytest.mark.parametrize("n,sc,lsc", [(48, 1, 3), (212, 2, 8), (752, 3, 10), (212, 6, 20)])
def test_gpu_logmap_siso_vs_unpinned_oracle_and_exact(n, sc, lsc):
    """The GPU SISO against the oracle with correctly rounded primitives (not the
    device's tables): the only difference is the instructions' 1-ulp deviations,
    so within 4e-6 + 2 ulp(M); and against exact f64 log-MAP within the SISO bound."""
    _gpu()
    O.set_trans(None)
    rng = np.random.default_rng(3 * n + lsc)
    Lc = (rng.standard_normal((4, 2, n)) * sc).astype(np.float32)
    La = rng.standard_normal((2, 2, n)) * lsc
    A, B = M.bcjr_max_log_map_batch(*Lc, *La, *TAB, n, 0.7, algo="log-map")
    for b in range(2):
        lc, la = Lc[:, b], La[:, b]
        UA, UB = O.siso(*lc, *la, TAB, 0.7, algo=1)
        big = max(np.max(np.abs(lc[0] + la[0])), np.max(np.abs(lc[1] + la[1])), 1.0)
        tight = 4e-6 + 2 * float(np.spacing(np.float32(big)))
        assert max(np.max(np.abs(A[b] - UA)), np.max(np.abs(B[b] - UB))) <= tight
        RA, RB = O.siso(*lc, *la, TAB, 0.7, algo=2)
        assert max(np.max(np.abs(A[b] - RA)), np.max(np.abs(B[b] - RB))) <= _siso_tol(lc, la)
