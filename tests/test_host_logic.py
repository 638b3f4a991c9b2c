"""Host-side logic of the drop-in API (no GPU): tables, the de-puncture walk,
error behaviour of the constructor, the demapper's dtype rules, the host
encoder -- all against the reference's golden vectors."""
import numpy as np
import pytest

from modulations_amd import demap as D
from modulations_amd import dvb_rcs2_turbo as M
from modulations_amd import tables as T


def test_constructor_errors():
    with pytest.raises(ValueError):
        M.DVBRCS2_Turbo(1504, "1/3")          # N counts couples: SURVEY fact 9, :295-296
    with pytest.raises(KeyError):
        M.DVBRCS2_Turbo(752, "5/6")           # :292


def test_codec_attributes(G_tables):
    c = M.DVBRCS2_Turbo(752, "1/3")
    assert c.k_info == 1504 and c.n_coded == 4512 and c.iterations == 8
    assert np.array_equal(c.perm, G_tables["perm_752"])
    assert np.array_equal(c.inv_perm, np.argsort(c.perm).astype(np.int32))   # the reference's :325 on this host
    assert np.array_equal(M.DVBRCS2_Turbo(752, "1/3", inv_perm="stable").inv_perm, G_tables["inv_stable_752"])
    for k in ("next_state", "out_W", "out_Y", "prev_state", "prev_input"):
        assert np.array_equal(getattr(c, k), G_tables[k])
    assert np.array_equal(c.G_matrix, G_tables["G"])
    assert M.DVBRCS2_Turbo(752, "1/2").n_coded == 3008


def test_numpy_inverse_mode_matches_reference_expression(G_tables):
    c = M.DVBRCS2_Turbo(48, "1/3", inv_perm="numpy")
    assert np.array_equal(c.inv_perm, np.argsort(c.perm).astype(np.int32))


def test_gf2_helpers(G_tables):
    for n in (48, 212, 752):
        gp = M.mat_pow_gf2(G_tables["G"], n)
        assert np.array_equal(gp, G_tables[f"gpow_{n}"])
        assert [M.solve_circular_state_gf2(gp, z) for z in range(16)] == list(G_tables[f"circ_{n}"])
    assert M.max_star(1.0, 2.0) == 2.0 and M.max_star(3.0, 2.0) == 3.0


def test_host_encode_matches_reference(G_encode):
    for k in G_encode.files:
        if not k.startswith("bits_"):
            continue
        key = k[5:]
        n, r1, r2 = key.split("_")
        c = M.DVBRCS2_Turbo(int(n), f"{r1}/{r2}")
        for b, cw in zip(G_encode[k][:2], G_encode[f"coded_{key}"][:2]):
            assert np.array_equal(c.encode(b), cw)


@pytest.mark.parametrize("n", [48, 64, 212, 220, 424, 752, 848])
@pytest.mark.parametrize("rate", ["1/3", "1/2", "2/3", "3/4"])
def test_compiled_host_encode_matches_oracle(n, rate):
    """DVBRCS2_Turbo.encode / encode_batch run tdec_encode_host (compiled, no
    GPU): equal to the oracle's restatement of :404-462 for random rows, the
    reference's extra-bits and index-wrap behaviour kept."""
    from oracle import oracle as O
    c = M.DVBRCS2_Turbo(n, rate)
    t, G = O.trellis()
    pm = T.puncture_matrix(c.punct)
    rng = np.random.default_rng(n)
    info = rng.integers(0, 2, (5, c.k_info)).astype(np.int32)
    got = c.encode_batch(info)
    for b in range(5):
        assert np.array_equal(got[b], O.encode(info[b], n, c.punct["period"], pm, c.perm, t, G))
        assert np.array_equal(c.encode(info[b]), got[b])
    assert np.array_equal(c.encode(np.concatenate([info[0], [1, 0, 1]])), got[0])   # extra bits ignored
    with pytest.raises(IndexError):
        c.encode(info[0][:-2])
    bad = info[0].copy()
    bad[4] = 2                                       # (2 << 1) | B = 4: numpy IndexError
    with pytest.raises(IndexError):
        c.encode(bad)


@pytest.mark.parametrize("rate", ["1/3", "1/2", "2/3", "3/4"])
def test_puncture_walk(rate):
    p = T.PUNCTURE_PATTERNS[rate]
    for n in (48, 212, 752):
        consumed = T.consumed_size(n, p)
        assert consumed >= T.coded_size(n, p)
        if n % p["period"] == 0:
            assert consumed == T.coded_size(n, p)


def test_rate_two_thirds_quirk():
    """rate 2/3 with N % 3 != 0 reads more LLRs than n_coded (:398-402)."""
    p = T.PUNCTURE_PATTERNS["2/3"]
    assert T.coded_size(64, p) == 189 and T.consumed_size(64, p) == 192


def test_demap_dtype_rules():
    # QPSK's constellation is complex128 -> f64 arithmetic (qpsk_mod divides by np.sqrt(2))
    assert D.constellation("QPSK").dtype == np.complex128
    assert D.demap_mode(np.complex64, np.complex128, np.float64(0.1)) == (True, False, 0.1)
    # complex64 arithmetic, np.float64 noise var -> f64 division (the call site, :464-471)
    assert D.demap_mode(np.complex64, np.complex64, np.float64(0.1))[:2] == (False, False)
    # Python float -> numpy >= 2 keeps float32 (NEP 50); the 0.005 floor is a Python float
    assert D.demap_mode(np.complex64, np.complex64, 0.1)[:2] == (False, True)
    assert D.demap_mode(np.complex64, np.complex64, np.float64(0.001)) == (False, True, 0.005)


def test_valid_interleaver_is_permutation():
    for n in T.INTERLEAVER_PARAMS:
        assert sorted(T.valid_interleaver(n)) == list(range(n))
        assert len(np.unique(T.interleaver(n))) < n          # the reference's is not


def test_legacy_codec_shim():
    """turbo_test_suite.py / test_sdr_with_coding.py construct DVB_RCS2_TurboCodec
    with keywords and read code_rate as a float (turbo_test_suite.py:133)."""
    c = M.DVB_RCS2_TurboCodec(block_length=212, code_rate='1/2', n_iterations=10)
    assert c.N == 212 and c.k_info == 424 and c.n_coded == 848 and c.iterations == 10
    assert c.code_rate == 0.5 and c.block_length == 212 and c.n_iterations == 10
    with pytest.raises(KeyError):
        M.DVB_RCS2_TurboCodec(block_length=212, code_rate='2/5')    # in the harness menu, not in the tables
    with pytest.raises(ValueError):
        M.DVB_RCS2_TurboCodec(block_length=228, code_rate='1/3')


def test_numpy_avx512_inverse_is_a_pinned_argsort(G_tables):
    """inv_perm='numpy-avx512' reproduces the reference's np.argsort(perm) as the
    survey's AVX-512 numpy 2.2 host evaluated it, on any host."""
    from modulations_amd import tables as T
    for n in (48, 64, 212, 220, 424, 752, 848):
        perm = T.interleaver(n)
        inv = T.inverse_interleaver(perm, "numpy-avx512")
        assert np.array_equal(inv, G_tables[f"inv_default_{n}"])
        assert sorted(inv.tolist()) == list(range(n))            # a permutation
        assert np.all(np.diff(perm[inv]) >= 0)                   # that sorts perm
    with pytest.raises(ValueError):
        T.inverse_interleaver(T.valid_interleaver(48), "numpy-avx512")
