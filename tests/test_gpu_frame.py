"""The frame decoder (csrc/tdec_frame.hip): one codeword per workgroup, the
recursions split into 4 segments per direction that re-run from their
predecessor's end vector until they merge with the stored trajectory.  It serves
bcjr_max_log_map / bcjr_decode_circular (every row of a call) and small
decode batches.  Every case is compared with the C oracle (the restatement of
dvb_rcs2_turbo.py:116-281 / :464-537 pinned to the reference's golden vectors)
by IEEE == (NaN == NaN where the reference produces NaN).

The segment machinery is exact only if the merge test and the re-run rounds
are right, so the inputs below also include the cases that defeat early
merging: NaN / inf LLRs (a NaN vector never equals the stored one: every
segment runs to its end and hands its vector on), tiny LLRs (long mixing),
lengths that leave empty or short segments (N = 1 .. 17) and lengths that are
not multiples of 4."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


TAB, _ = O.trellis()
_REF = M.DVBRCS2_Turbo(48, "1/3")
TABLES = (_REF.next_state, _REF.out_W, _REF.out_Y, _REF.prev_state, _REF.prev_input)


def _siso_inputs(rng, B, n, lc_scale, la_scale):
    Lc = [(rng.standard_normal((B, n)) * lc_scale).astype(np.float32) for _ in range(4)]
    La = [rng.standard_normal((B, n)) * la_scale for _ in range(2)]
    return Lc, La


def _check_siso(Lc, La, n, sf):
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *TABLES, n, sf)
    for b in range(Lc[0].shape[0]):
        rA, rB = O.siso(Lc[0][b], Lc[1][b], Lc[2][b], Lc[3][b], La[0][b], La[1][b], TAB, sf)
        np.testing.assert_array_equal(LeA[b], rA)
        np.testing.assert_array_equal(LeB[b], rB)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 33, 48, 64, 100, 212, 220, 424, 752, 790, 848,
                               1010, 1100])
@pytest.mark.parametrize("sf", [0.7, 1.0])
def test_frame_siso_matches_oracle(n, sf):
    rng = np.random.default_rng(n * 7 + int(sf * 10))
    Lc, La = _siso_inputs(rng, 3, n, 3.0, 8.0)
    _check_siso(Lc, La, n, sf)


@pytest.mark.parametrize("wpd", ["one", "two"])
def test_frame_siso_every_length_to_160(wpd, monkeypatch):
    """Every N from 1 to 160 (segments per direction N / 32, split evenly in whole
    4-step blocks, ragged last blocks, 8-step fast blocks and their per-step tail)
    on both recursion layouts (TDEC_FR_SISO_WPD1_MAX: one wave per direction, or
    two), at a low a-priori scale so merges come late and rounds hand end vectors
    down the chain."""
    if wpd == "two":
        monkeypatch.setenv("TDEC_FR_SISO_WPD1_MAX", "0")
    rng = np.random.default_rng(160)
    for n in range(1, 161):
        Lc, La = _siso_inputs(rng, 2, n, 1.0, 1.0)
        _check_siso(Lc, La, n, 0.7)


def test_frame_siso_single_row_is_the_drop_in():
    rng = np.random.default_rng(3)
    n = 752
    Lc, La = _siso_inputs(rng, 1, n, 2.0, 5.0)
    a, b = M.bcjr_decode_circular(*(x[0] for x in Lc), *(x[0] for x in La), *TABLES, n, 0.7)
    rA, rB = O.siso(*(x[0] for x in Lc), *(x[0] for x in La), TAB, 0.7)
    np.testing.assert_array_equal(a, rA)
    np.testing.assert_array_equal(b, rB)


@pytest.mark.parametrize("n", [5, 48, 212, 752])
@pytest.mark.parametrize("kind", ["zeros", "tiny", "huge", "nan", "inf", "mixed", "denormal", "ties"])
def test_frame_siso_adversarial(n, kind):
    rng = np.random.default_rng(sum(map(ord, kind)) + n)
    B = 2
    Lc, La = _siso_inputs(rng, B, n, 2.0, 4.0)
    if kind == "zeros":
        Lc = [np.zeros_like(x) for x in Lc]
        La = [np.zeros_like(x) for x in La]
    elif kind == "tiny":
        Lc = [(x * 1e-4).astype(np.float32) for x in Lc]
        La = [x * 1e-5 for x in La]
    elif kind == "huge":
        Lc = [(x * 1e6).astype(np.float32) for x in Lc]
        La = [x * 1e12 for x in La]
    elif kind == "nan":
        for x in Lc + La:
            x[:, rng.integers(0, n, max(1, n // 10))] = np.nan
    elif kind == "inf":
        for i, x in enumerate(Lc + La):
            x[:, rng.integers(0, n, max(1, n // 10))] = np.inf if i % 2 else -np.inf
    elif kind == "mixed":
        Lc[0][0, :] = np.nan
        Lc[2][1, n // 2] = np.inf
        La[1][1, 0] = -np.inf
    elif kind == "denormal":
        Lc = [(x * 1e-42).astype(np.float32) for x in Lc]
        La = [x * 1e-310 for x in La]
    elif kind == "ties":
        Lc = [np.sign(x).astype(np.float32) for x in Lc]
        La = [np.zeros_like(x) for x in La]
    _check_siso(Lc, La, n, 0.7)


@pytest.mark.parametrize("n,rate", [(48, "1/3"), (64, "3/4"), (212, "1/3"), (220, "2/3"), (424, "1/2"),
                                    (752, "1/3"), (752, "1/2"), (848, "1/3"), (848, "1/2")])
@pytest.mark.parametrize("B,noise", [(1, 0.8), (2, 2.5), (65, 1.6)])
def test_frame_decode_matches_oracle(n, rate, B, noise):
    rng = np.random.default_rng(n + B)
    c = M.DVBRCS2_Turbo(n, rate)
    info = rng.integers(0, 2, (B, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in info]).astype(np.float32)
    llr += (rng.standard_normal(llr.shape) * noise).astype(np.float32)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, TAB, want_lfinal=True, nthreads=8)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)


@pytest.mark.parametrize("n,rate", [(48, "1/3"), (212, "1/3"), (424, "1/2"), (752, "1/3"), (848, "1/3")])
@pytest.mark.parametrize("layout", ["one", "two"])
def test_frame_decode_both_recursion_layouts(n, rate, layout, monkeypatch):
    """The decoder with one wave per recursion direction and with two, at every
    block size, whatever tdec_api.hip fr_wpd would pick (TDEC_FR_WPD1_MAX, read per
    call): the same bits and L_final as the oracle."""
    monkeypatch.setenv("TDEC_FR_WPD1_MAX", "100000" if layout == "one" else "0")
    rng = np.random.default_rng(n + 7)
    c = M.DVBRCS2_Turbo(n, rate)
    B = 33
    info = rng.integers(0, 2, (B, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in info]).astype(np.float32)
    llr += (rng.standard_normal(llr.shape) * 1.7).astype(np.float32)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, TAB, want_lfinal=True, nthreads=8)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)


@pytest.mark.parametrize("kind", ["nan", "inf", "tiny"])
@pytest.mark.parametrize("n", [212, 848])
def test_frame_decode_nonfinite_and_tiny(kind, n):
    """(N = 848: the frame decoder with Le2 in global scratch, tdec_frame.hip fr_lds)"""
    rng = np.random.default_rng(11)
    c = M.DVBRCS2_Turbo(n, "1/3")
    llr = (rng.standard_normal((3, c.n_coded)) * 2).astype(np.float32)
    if kind == "nan":
        llr[0, rng.integers(0, c.n_coded, 20)] = np.nan
        llr[2, :] = np.nan
    elif kind == "inf":
        llr[0, rng.integers(0, c.n_coded, 20)] = np.inf
        llr[1, rng.integers(0, c.n_coded, 20)] = -np.inf
    else:
        llr *= np.float32(1e-4)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, TAB, want_lfinal=True, nthreads=8)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)


def test_frame_decode_valid_perm_round_trip():
    c = M.DVBRCS2_Turbo(752, "1/3", interleaver="valid-perm")
    rng = np.random.default_rng(4)
    info = rng.integers(0, 2, (4, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * 20.0 for b in info]).astype(np.float32)
    assert np.array_equal(c.decode_batch(llr), info)


def test_frame_decode_n848_batches_and_lfinal_every_row():
    """N = 848 (a reference block size, dvb_rcs2_turbo.py:12-17): the frame decoder's
    LDS plan is over 160 KiB there, so Le2 lives in global scratch; batches up to
    the routing limit, every row against the oracle."""
    rng = np.random.default_rng(848)
    c = M.DVBRCS2_Turbo(848, "1/3")
    B = 600
    base = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in rng.integers(0, 2, (16, c.k_info))])
    llr = (base[rng.integers(0, 16, B)] + rng.standard_normal((B, c.n_coded)) * 1.4).astype(np.float32)
    for rows in (slice(0, 1), slice(0, 64), slice(0, B)):
        bits, lf = c.decode_batch(llr[rows], return_lfinal=True)
        rb, rl = O.decode_batch(llr[rows], c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                                c.inv_perm, TAB, want_lfinal=True, nthreads=16)
        assert np.array_equal(bits, rb)
        np.testing.assert_array_equal(lf, rl)


@pytest.mark.parametrize("n,rate,B", [(752, "1/2", 12288), (212, "1/3", 8192)])
def test_frame_decode_at_the_routing_threshold(n, rate, B):
    """The frame decoder's batch limits (tdec_api.hip lowlat_max: 12 288 codewords
    for N >= 400, 8 192 below): the largest batches it serves, one workgroup each."""
    rng = np.random.default_rng(B + n)
    c = M.DVBRCS2_Turbo(n, rate)
    base = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in rng.integers(0, 2, (64, c.k_info))])
    llr = (base[rng.integers(0, 64, B)] + rng.standard_normal((B, c.n_coded)) * 1.6).astype(np.float32)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, TAB, want_lfinal=True, nthreads=16)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)
