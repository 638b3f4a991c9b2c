"""Hypothesis property tests of the HIP path against the oracle (SURVEY §4
item 4): random block lengths, batch sizes (ragged last tile, several tiles),
LLR scales from 1e-3 to 1e4, rates and both algorithms, bit for bit through
the C ABI.  Bounded example counts keep the run to seconds."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("trans_tables")]

from oracle import oracle as O  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402

SETTINGS = settings(max_examples=20, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _tabs():
    return T.trellis_tables()[:5]


@SETTINGS
@given(n=st.sampled_from([48, 64, 212, 220]), rate=st.sampled_from(["1/3", "1/2", "2/3", "3/4"]),
       B=st.integers(1, 140), scale=st.floats(1e-3, 1e4), it=st.integers(1, 8),
       algo=st.sampled_from(["max-log", "log-map"]), seed=st.integers(0, 2**31 - 1))
def test_decode_matches_oracle(n, rate, B, scale, it, algo, seed):
    c = M.DVBRCS2_Turbo(n, rate, iterations=it, algo=algo)
    llr = (np.random.default_rng(seed).standard_normal((B, T.consumed_size(n, c.punct))) * scale).astype(np.float32)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    t, _ = O.trellis()
    rows = [0, B // 2, B - 1]
    rb, rl = O.decode_batch(llr[rows], n, c.punct["period"], T.puncture_matrix(c.punct), it, c.perm, c.inv_perm,
                            t, algo=1 if algo == "log-map" else 0, want_lfinal=True)
    assert np.array_equal(bits[rows], rb) and np.array_equal(lf[rows], rl)


@SETTINGS
@given(n=st.integers(1, 300), B=st.integers(1, 130), scale=st.floats(1e-3, 1e4), la_scale=st.floats(0.0, 300.0),
       sf=st.sampled_from([0.7, 1.0]), algo=st.sampled_from(["max-log", "log-map"]), seed=st.integers(0, 2**31 - 1))
def test_siso_matches_oracle(n, B, scale, la_scale, sf, algo, seed):
    rng = np.random.default_rng(seed)
    Lc = (rng.standard_normal((4, B, n)) * scale).astype(np.float32)
    La = rng.standard_normal((2, B, n)) * la_scale
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), n, sf, algo=algo)
    t, _ = O.trellis()
    for b in {0, B // 2, B - 1}:
        rA, rB = O.siso(*Lc[:, b], *La[:, b], t, sf, algo=1 if algo == "log-map" else 0)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB), b


@SETTINGS
@given(n=st.integers(1, 1100), scale=st.floats(1e-3, 1e4), la_scale=st.floats(0.0, 300.0),
       sf=st.sampled_from([0.7, 1.0]), dt=st.sampled_from(["f32", "f64", "mixed", "int"]),
       algo=st.sampled_from(["max-log", "log-map"]), seed=st.integers(0, 2**31 - 1))
def test_single_call_siso_dtypes_match_oracle(n, scale, la_scale, sf, dt, algo, seed):
    """One bcjr_max_log_map call (the staged per-call path) or one-row batch
    (log-MAP) with the channel LLRs in each dtype numba specialises on
    (float32; float64; a mix, widened; integers), against the oracle's same
    specialisation, every extrinsic."""
    rng = np.random.default_rng(seed)
    Lc = [rng.standard_normal(n) * scale + 1e-9 for _ in range(4)]
    if dt == "f32":
        Lc = [x.astype(np.float32) for x in Lc]
    elif dt == "mixed":
        Lc[1], Lc[3] = Lc[1].astype(np.float32), Lc[3].astype(np.float32)
    elif dt == "int":
        Lc = [np.rint(x).astype(np.int64) for x in Lc]
    La = [rng.standard_normal(n) * la_scale for _ in range(2)]
    if algo == "max-log":
        LeA, LeB = M.bcjr_max_log_map(*Lc, *La, *_tabs(), n, sf)
    else:
        A, B = M.bcjr_max_log_map_batch(*(x[None] for x in Lc), *(x[None] for x in La), *_tabs(), n, sf, algo=algo)
        LeA, LeB = A[0], B[0]
    t, _ = O.trellis()
    rA, rB = O.siso(*Lc, *La, t, sf, algo=1 if algo == "log-map" else 0)
    np.testing.assert_array_equal(LeA, rA)
    np.testing.assert_array_equal(LeB, rB)
