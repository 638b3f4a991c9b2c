"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and the C oracle, bit-exact (IEEE ==) for max-log-MAP, demapper and
encoder; log-MAP within the stated tolerance.

Sizes stay small enough that the oracle finishes in seconds; the full-size
bench configuration is covered by size-independent properties
(tests/test_gpu_properties.py).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("trans_tables")]

from oracle import oracle as O  # noqa: E402
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402

RATES = ("1/3", "1/2", "2/3", "3/4")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _tabs():
    nx, ow, oy, ps, pi, _ = T.trellis_tables()
    return nx, ow, oy, ps, pi


def _awgn_llrs(rng, codec, B, ebn0_db, rate):
    """QPSK over AWGN with the decoder's sign (SURVEY §8 d)."""
    info = rng.integers(0, 2, (B, codec.k_info)).astype(np.int32)
    t, G = O.trellis()
    pm = T.puncture_matrix(codec.punct)
    coded = np.stack([O.encode(b, codec.N, codec.punct["period"], pm, codec.perm, t, G) for b in info])
    n0 = 1.0 / (rate * 2 * 10 ** (ebn0_db / 10.0))
    x = (1 - 2.0 * coded) / np.sqrt(2)
    y = x + np.sqrt(n0 / 2) * rng.standard_normal(x.shape)
    llr = (2 * np.sqrt(2) * y / n0).astype(np.float32)
    if llr.shape[1] < T.consumed_size(codec.N, codec.punct):
        llr = np.pad(llr, ((0, 0), (0, T.consumed_size(codec.N, codec.punct) - llr.shape[1])))
    return info, llr


# ---------------------------------------------------------------- SISO -------------
@pytest.mark.parametrize("n", [48, 212, 752])
def test_siso_golden(G_siso, n):
    g = G_siso
    for j in range(g[f"LcA_{n}"].shape[0]):
        LeA, LeB = M.bcjr_max_log_map(g[f"LcA_{n}"][j], g[f"LcB_{n}"][j], g[f"LcW_{n}"][j], g[f"LcY_{n}"][j],
                                      g[f"LaA_{n}"][j], g[f"LaB_{n}"][j], *_tabs(), n, g[f"sf_{n}"][j])
        assert np.array_equal(LeA, g[f"LeA_{n}"][j]), (n, j)
        assert np.array_equal(LeB, g[f"LeB_{n}"][j]), (n, j)


def test_siso_alias_and_batch_vs_oracle():
    assert M.bcjr_decode_circular is M.bcjr_max_log_map
    rng = np.random.default_rng(3)
    n, B = 212, 131                                   # ragged batch: 2 full waves + 3 lanes
    Lc = (rng.standard_normal((4, B, n)) * rng.uniform(0.3, 30, (1, B, 1))).astype(np.float32)
    La = rng.standard_normal((2, B, n)) * 40
    t, _ = O.trellis()
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), n, 0.7)
    for b in range(B):
        rA, rB = O.siso(Lc[0, b], Lc[1, b], Lc[2, b], Lc[3, b], La[0, b], La[1, b], t, 0.7)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB), b


def test_siso_extreme_inputs():
    """Huge / tiny / signed-zero inputs: the -1e9 floor, the +-300 clip and denormals."""
    t, _ = O.trellis()
    n = 48
    cases = [np.full((4, n), 1e12, np.float32), np.full((4, n), -3e8, np.float32),
             np.full((4, n), 1e-40, np.float32), np.full((4, n), -0.0, np.float32)]
    rng = np.random.default_rng(0)
    mixed = (rng.standard_normal((4, n)) * 10).astype(np.float32)
    mixed[:, ::5] = 2e9
    cases.append(mixed)
    for Lc in cases:
        La = np.zeros((2, n))
        La[0, ::3] = 1e-310                            # f64 denormal a-priori
        LeA, LeB = M.bcjr_max_log_map(*Lc, *La, *_tabs(), n, 1.0)
        rA, rB = O.siso(*Lc, *La, t, 1.0)
        assert np.array_equal(LeA, rA) and np.array_equal(LeB, rB)


def test_logmap_extreme_inputs_take_both_first_maxstar_paths():
    """log-MAP recursions test all 16 first max* of a step at once (kernel
    acc_first16) and fall back to the per-state test when a candidate lies
    within 256 of the -1e9 floor.  Rows of one wave mix ordinary metrics with
    metrics at the floor (inputs of 1e9 scale), so both paths and the per-lane
    fallback run; SISO and full decode equal the oracle bit for bit."""
    t, _ = O.trellis()
    n, B = 48, 9
    rng = np.random.default_rng(5)
    Lc = (rng.standard_normal((4, B, n)) * 4).astype(np.float32)
    Lc[:, 0] = 1e12
    Lc[:, 1] = -3e8
    Lc[:, 2] = (np.sign(rng.standard_normal((4, n))) * 1e9).astype(np.float32)
    Lc[:, 3, ::4] = 2e9
    Lc[:, 4] = (rng.standard_normal((4, n)) * 5e8).astype(np.float32)
    Lc[:, 5, ::7] = -1.5e9
    Lc[:, 6] = np.float32(1e-40)
    La = rng.standard_normal((2, B, n)) * 10
    La[:, 7] = 3e8
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), n, 0.7, algo="log-map")
    for b in range(B):
        rA, rB = O.siso(*Lc[:, b], *La[:, b], t, 0.7, algo=1)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB), b
    c = M.DVBRCS2_Turbo(n, "1/3", algo="log-map")
    llr = (rng.standard_normal((B, c.n_coded)) * 3).astype(np.float32)
    llr[0] = 1e9
    llr[1, ::3] = -2e9
    llr[2] = (np.sign(rng.standard_normal(c.n_coded)) * 7e8).astype(np.float32)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = O.decode_batch(llr, n, c.punct["period"], T.puncture_matrix(c.punct), 8, c.perm, c.inv_perm, t,
                            algo=1, want_lfinal=True)
    assert np.array_equal(bits, rb) and np.array_equal(lf, rl)


# ---------------------------------------------------------------- decode -----------
def test_decode_golden(G_decode):
    keys = sorted(k[4:] for k in G_decode.files if k.startswith("llr_"))
    for key in keys:
        n, r1, r2, variant = key.split("_")
        c = M.DVBRCS2_Turbo(int(n), f"{r1}/{r2}", inv_perm=G_decode[f"inv_{key}"])
        bits, lf = c.decode_batch(G_decode[f"llr_{key}"], return_lfinal=True)
        assert np.array_equal(bits, G_decode[f"bits_{key}"]), key
        assert np.array_equal(lf, G_decode[f"lfinal_{key}"]), key
        # single-codeword drop-in call
        assert np.array_equal(c.decode(G_decode[f"llr_{key}"][0]), G_decode[f"bits_{key}"][0])


def test_decode_reference_host_default_fixtures(G_decode):
    """The *_default fixtures were decoded by the reference with its own
    inv_perm = np.argsort(perm) on the survey's AVX-512 host.  The drop-in
    reproduces them with the one-line switch inv_perm='numpy-avx512' (and with
    inv_perm='numpy' wherever this host's numpy sorts the same way)."""
    from modulations_amd import tables as T
    keys = sorted(k[4:] for k in G_decode.files if k.startswith("llr_") and k.endswith("_default"))
    assert keys
    for key in keys:
        n, r1, r2, _ = key.split("_")
        c = M.DVBRCS2_Turbo(int(n), f"{r1}/{r2}", inv_perm="numpy-avx512")
        assert np.array_equal(c.inv_perm, G_decode[f"inv_{key}"])
        bits, lf = c.decode_batch(G_decode[f"llr_{key}"], return_lfinal=True)
        assert np.array_equal(bits, G_decode[f"bits_{key}"]), key
        assert np.array_equal(lf, G_decode[f"lfinal_{key}"]), key
        if np.array_equal(T.inverse_interleaver(c.perm, "numpy"), G_decode[f"inv_{key}"]):
            c2 = M.DVBRCS2_Turbo(int(n), f"{r1}/{r2}", inv_perm="numpy")
            assert np.array_equal(c2.decode_batch(G_decode[f"llr_{key}"]), G_decode[f"bits_{key}"]), key


@pytest.mark.parametrize("n", [48, 212, 752])
def test_noise_free_kat(G_decode, n):
    """21 / 83 / 355 errors from the broken interleaver."""
    c = M.DVBRCS2_Turbo(n, "1/3", inv_perm=G_decode[f"kat_inv_{n}"])
    info = G_decode[f"kat_info_{n}"]
    bits = c.decode((1 - 2 * c.encode(info)) * 20.0)
    assert np.array_equal(bits, G_decode[f"kat_bits_{n}"])
    assert int((bits != info).sum()) == {48: 21, 212: 83, 752: 355}[n]


@pytest.mark.parametrize("n,rate", [(48, "1/3"), (64, "1/2"), (212, "1/3"), (220, "3/4"), (424, "2/3"),
                                    (752, "1/3"), (752, "1/2"), (848, "1/3")])
def test_decode_vs_oracle(n, rate):
    rng = np.random.default_rng(n * 7 + len(rate))
    c = M.DVBRCS2_Turbo(n, rate)
    R = {"1/3": 1 / 3, "1/2": 1 / 2, "2/3": 2 / 3, "3/4": 3 / 4}[rate]
    B = 70 if n <= 212 else 20
    info, llr = _awgn_llrs(rng, c, B, rng.choice([0.0, 1.5, 3.0]), R)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    t, _ = O.trellis()
    rb, rl = O.decode_batch(llr, n, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, t, want_lfinal=True)
    assert np.array_equal(bits, rb)
    assert np.array_equal(lf, rl)


def test_decode_iterations_and_errors():
    rng = np.random.default_rng(11)
    t, _ = O.trellis()
    for it in (1, 2, 5):
        c = M.DVBRCS2_Turbo(48, "1/3", iterations=it)
        _, llr = _awgn_llrs(rng, c, 65, 1.0, 1 / 3)
        rb = O.decode_batch(llr, 48, 1, T.puncture_matrix(c.punct), it, c.perm, c.inv_perm, t)
        assert np.array_equal(c.decode_batch(llr), rb)
    c = M.DVBRCS2_Turbo(48, "1/3")
    with pytest.raises(IndexError):
        c.decode(np.zeros(c.n_coded - 1))            # the reference's de-puncture IndexError
    assert c.decode(np.zeros(c.n_coded + 5)).shape == (96,)   # extra LLRs are ignored
    c = M.DVBRCS2_Turbo(212, "2/3")   # period 3 does not divide N: n_coded (630) < the walk (636)
    with pytest.raises(IndexError):
        c.decode(np.zeros(c.n_coded))                # what the reference's receive chain hands decode()
    with pytest.raises(UnboundLocalError):
        M.DVBRCS2_Turbo(48, "1/3", iterations=0).decode(np.zeros(288))
    bad = list(_tabs())
    bad[0] = bad[0].copy()
    bad[0][0, 0] = 5
    with pytest.raises(ValueError):
        M.bcjr_max_log_map(*np.zeros((4, 48), np.float32), *np.zeros((2, 48)), *bad, 48, 1.0)


def test_turbo_decode_alias():
    rng = np.random.default_rng(5)
    c = M.DVBRCS2_Turbo(212, "1/2")
    _, llr = _awgn_llrs(rng, c, 3, 2.0, 0.5)
    assert np.array_equal(M.turbo_decode(llr[0], 212, "1/2"), c.decode(llr[0]))
    assert np.array_equal(M.turbo_decode(llr, 212, "1/2"), c.decode_batch(llr))


def test_decode_device_path_matches_host_path():
    rng = np.random.default_rng(8)
    c = M.DVBRCS2_Turbo(752, "1/3")
    _, llr = _awgn_llrs(rng, c, 100, 1.0, 1 / 3)
    dl = torch.from_numpy(llr).cuda()
    bits = c.decode_device(dl)
    torch.cuda.synchronize()
    assert np.array_equal(bits.cpu().numpy(), c.decode_batch(llr))


def test_valid_perm_mode_decodes_clean_channel():
    rng = np.random.default_rng(2)
    c = M.DVBRCS2_Turbo(752, "1/3", interleaver="valid-perm")
    info = rng.integers(0, 2, (4, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * 20 for b in info])
    assert np.array_equal(c.decode_batch(llr), info)


# ---------------------------------------------------------------- log-MAP ----------
def test_logmap_vs_oracle():
    """Build-defined log-MAP.  max* is defined as a fixed f32
    operation sequence that both the kernel and the oracle restate, so it is
    bit-exact too (the north-star tolerance of 1e-5 is not needed)."""
    rng = np.random.default_rng(21)
    t, _ = O.trellis()
    for n, rate, R, B in ((752, "1/2", 0.5, 4), (212, "1/3", 1 / 3, 8)):
        c = M.DVBRCS2_Turbo(n, rate, algo="log-map")
        _, llr = _awgn_llrs(rng, c, B, 1.0, R)
        bits, lf = c.decode_batch(llr, return_lfinal=True)
        rb, rl = O.decode_batch(llr, n, c.punct["period"], T.puncture_matrix(c.punct), 8, c.perm, c.inv_perm, t,
                                algo=1, want_lfinal=True)
        assert np.array_equal(lf, rl) and np.array_equal(bits, rb)
    Lc = (rng.standard_normal((4, 5, 212)) * 4).astype(np.float32)
    La = rng.standard_normal((2, 5, 212)) * 10
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), 212, 0.7, algo="log-map")
    for b in range(5):
        rA, rB = O.siso(Lc[0, b], Lc[1, b], Lc[2, b], Lc[3, b], La[0, b], La[1, b], t, 0.7, algo=1)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB)


# ---------------------------------------------------------------- demapper ---------
@pytest.mark.parametrize("mod", ["BPSK", "QPSK", "8PSK", "16QAM"])
def test_demap_golden(G_demap, mod):
    g = G_demap
    syms = g[f"syms_{mod}"]
    assert np.array_equal(D.compute_llr(syms, mod, np.float64(0.137)), g[f"llr_f64nv_{mod}"])
    assert np.array_equal(D.compute_llr(syms, mod, np.float64(0.001)), g[f"llr_f64nvsmall_{mod}"])
    assert np.array_equal(D.compute_llr(syms, mod, 0.02), g[f"llr_pyfloat_{mod}"])
    assert np.array_equal(D.compute_llr(syms.astype(np.complex128) * (1 + 1e-9), mod, np.float64(0.2)),
                          g[f"llr_c128_{mod}"])


@pytest.mark.parametrize("mod", ["64QAM", "256QAM"])
def test_demap_high_order_vs_oracle(mod):
    rng = np.random.default_rng(4)
    cons = D.constellation(mod)
    syms = (cons[rng.integers(0, len(cons), 3000)] +
            0.05 * (rng.standard_normal(3000) + 1j * rng.standard_normal(3000))).astype(np.complex64)
    syms[:3] = [np.nan, np.inf, 0]
    bps = D.MODULATIONS[mod]["bps"]
    for nv in (np.float64(0.02), 0.3):
        f64, div32, nve = D.demap_mode(syms.dtype, cons.dtype, nv)
        ref = O.demap(syms, cons, bps, nve, div_f32=div32)
        assert np.array_equal(D.compute_llr(syms, mod, nv), ref, equal_nan=True)
        assert np.array_equal(D.compute_llr(syms, mod, nv, sign=-1), -ref, equal_nan=True)


def _adversarial_symbols(cons, rng, n):
    """Symbols that stress the separable-QAM candidate search: exactly on points,
    on decision bisectors (exact ties), within a few ulp of a bisector, far
    outside the grid, tiny, huge, NaN/inf, plus noisy points."""
    lv = np.unique(cons.real.astype(np.float64))
    mids = (lv[:-1] + lv[1:]) / 2
    pts = [cons[rng.integers(0, len(cons), n)] + 0.3 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)),
           cons[rng.integers(0, len(cons), 50)],
           rng.choice(mids, 50) + 1j * rng.choice(lv, 50),
           rng.choice(lv, 50) + 1j * rng.choice(mids, 50),
           rng.choice(mids, 50) + 1j * rng.choice(mids, 50),
           np.nextafter(rng.choice(mids, 50), 9) + 1j * np.nextafter(rng.choice(mids, 50), -9),
           (rng.choice(mids, 50) + 1e-7) + 1j * rng.choice(lv, 50),
           10 * (rng.standard_normal(50) + 1j * rng.standard_normal(50)),
           1e-20 * (rng.standard_normal(20) + 1j * rng.standard_normal(20)),
           np.array([0, 1e30, -1e30j, 3e38 + 3e38j, np.nan, np.inf, -np.inf + 1j, 1 + np.nan * 1j])]
    return np.concatenate(pts)


@pytest.mark.parametrize("mod", ["16QAM", "64QAM", "256QAM"])
@pytest.mark.parametrize("dt", [np.complex64, np.complex128])
def test_demap_separable_qam_adversarial(mod, dt):
    """The per-axis candidate search (k_demap/k_demap_planes on square QAM) must
    equal the full scan of compute_llr bit for bit, near-ties included."""
    rng = np.random.default_rng(12)
    cons = D.constellation(mod)
    syms = _adversarial_symbols(cons, rng, 4000).astype(dt)
    bps = D.MODULATIONS[mod]["bps"]
    for nv in (np.float64(0.05), 0.01):
        f64, div32, nve = D.demap_mode(syms.dtype, cons.dtype, nv)
        ref = O.demap(syms, cons, bps, nve, div_f32=div32)
        got = D.compute_llr(syms, mod, nv)
        assert np.array_equal(got, ref, equal_nan=True)
    # the device tensor path and the fused planes path share the device code
    dev = D.compute_llr_device(torch.from_numpy(syms).cuda(), mod, np.float64(0.05))
    torch.cuda.synchronize()
    _, div32, nve = D.demap_mode(syms.dtype, cons.dtype, np.float64(0.05))
    assert np.array_equal(dev.cpu().numpy(), O.demap(syms, cons, bps, nve, div_f32=div32), equal_nan=True)


def test_demap_device_tensor():
    rng = np.random.default_rng(6)
    cons = D.constellation("16QAM")
    syms = (cons[rng.integers(0, 16, 5000)] + 0.2 * rng.standard_normal(5000)).astype(np.complex64)
    out = D.compute_llr_device(torch.from_numpy(syms).cuda(), "16QAM", np.float64(0.1))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), O.demap(syms, cons, 4, 0.1))


@pytest.mark.parametrize("mod,n,rate", [("16QAM", 752, "1/3"), ("8PSK", 752, "1/2"), ("QPSK", 212, "1/3"),
                                        ("256QAM", 752, "1/3")])
def test_fused_demap_planes_decode_vs_host_chain(mod, n, rate):
    """demap -> (pad/truncate to n_coded, :474-478) -> f32 -> decode, fused on the
    device, equals compute_llr (decoder sign) followed by decode()."""
    rng = np.random.default_rng(31)
    c = M.DVBRCS2_Turbo(n, rate)
    bps = D.MODULATIONS[mod]["bps"]
    cons = D.constellation(mod)
    B = 67
    S = -(-c.n_coded // bps)
    syms = (cons[rng.integers(0, len(cons), (B, S))] +
            0.15 * (rng.standard_normal((B, S)) + 1j * rng.standard_normal((B, S)))).astype(np.complex64)
    nv = np.float64(0.0225)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, nv)
    planes = torch.empty(c.planes_bytes(B) // 4, dtype=torch.float32, device="cuda")
    bits = torch.empty((B, c.k_info), dtype=torch.int32, device="cuda")
    c.reserve(B)
    c.demap_planes_device(torch.from_numpy(syms).cuda(), cons, bps, nve, planes, div_f32=div32)
    c.decode_planes_device(planes, B, bits)
    torch.cuda.synchronize()
    llr = np.stack([-O.demap(s, cons, bps, nve, div_f32=div32)[:c.n_coded] for s in syms]).astype(np.float32)
    t, _ = O.trellis()
    rb = O.decode_batch(llr, n, c.punct["period"], T.puncture_matrix(c.punct), 8, c.perm, c.inv_perm, t)
    assert np.array_equal(bits.cpu().numpy(), rb)


# ---------------------------------------------------------------- encoder ----------
@pytest.mark.parametrize("n,rate", [(48, "1/3"), (212, "1/2"), (752, "1/3"), (48, "3/4"), (64, "2/3")])
def test_device_encoder(G_encode, n, rate):
    c = M.DVBRCS2_Turbo(n, rate)
    rng = np.random.default_rng(n)
    info = rng.integers(0, 2, (150, c.k_info)).astype(np.uint8)
    out = c.encode_device(torch.from_numpy(info).cuda())
    torch.cuda.synchronize()
    t, G = O.trellis()
    pm = T.puncture_matrix(c.punct)
    for b in range(0, 150, 7):
        ref = O.encode(info[b].astype(np.int32), n, c.punct["period"], pm, c.perm, t, G)
        assert np.array_equal(out[b].cpu().numpy().astype(np.int32), ref)
    key = f"{n}_{rate.replace('/', '_')}"
    if f"bits_{key}" in G_encode.files:
        gb = torch.from_numpy(G_encode[f"bits_{key}"].astype(np.uint8)).cuda()
        assert np.array_equal(c.encode_device(gb).cpu().numpy(), G_encode[f"coded_{key}"])


def test_legacy_codec_shim_decodes_like_the_codec():
    """The BPSK AWGN recipe of turbo_test_suite.py:128-161 through the legacy name."""
    rng = np.random.default_rng(12)
    c = M.DVB_RCS2_TurboCodec(block_length=212, code_rate='1/3', n_iterations=8)
    ref = M.DVBRCS2_Turbo(212, '1/3', 8)
    snr = 10 ** (1.0 / 10)
    nv = 1.0 / (2.0 * c.code_rate * snr)
    for _ in range(3):
        info = rng.integers(0, 2, c.k_info)
        y = 1.0 - 2.0 * c.encode(info).astype(float) + np.sqrt(nv) * rng.standard_normal(c.n_coded)
        llr = np.clip(2.0 * y / nv, -50, 50)
        assert np.array_equal(c.decode(llr), ref.decode(llr))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 50, 213])
@pytest.mark.parametrize("algo", ["max-log", "log-map"])
def test_siso_any_block_length(n, algo):
    """bcjr_max_log_map accepts any N (the reference loops over range(N)); the
    kernel's ragged top window must match the oracle bit for bit."""
    rng = np.random.default_rng(n)
    B = 70
    Lc = (rng.standard_normal((4, B, n)) * 3).astype(np.float32)
    La = rng.standard_normal((2, B, n)) * 6
    t, _ = O.trellis()
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), n, 0.7, algo=algo)
    for b in range(0, B, 9):
        rA, rB = O.siso(Lc[0, b], Lc[1, b], Lc[2, b], Lc[3, b], La[0, b], La[1, b], t, 0.7,
                        algo=1 if algo == "log-map" else 0)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB), b


def test_decode_ragged_block_length_through_c_abi():
    """A non-table N (50 couples, own bijective interleaver) through tdec_create /
    tdec_decode_batch: the ragged decode instantiation vs the oracle."""
    import ctypes
    from modulations_amd import _native as NT
    n = 50
    perm = ((7 * np.arange(n) + 3) % n).astype(np.int32)
    inv = np.argsort(perm).astype(np.int32)
    punct = T.PUNCTURE_PATTERNS["1/3"]
    h = M._Handle(0, n, punct, 8, 0, perm, inv, T.packed_tables(*_tabs()))
    rng = np.random.default_rng(50)
    llr = (rng.standard_normal((65, 6 * n)) * 3).astype(np.float32)
    bits = np.zeros((65, 2 * n), np.int32)
    NT.check(NT.lib().tdec_decode_batch(h.h, 65, NT.ptr(llr), 6 * n, NT.ptr(bits), None))
    t, _ = O.trellis()
    rb = O.decode_batch(llr, n, 1, T.puncture_matrix(punct), 8, perm, inv, t)
    assert np.array_equal(bits, rb)


def test_empty_batches_are_no_ops():
    """B = 0 through every batched entry point returns empty results, as numpy
    would for an empty leading axis; N = 0 SISO returns empty extrinsics, as the
    reference's recursions over range(0) do; B < 0 is rejected."""
    import ctypes
    from modulations_amd import _native as NT
    c = M.DVBRCS2_Turbo(212, "1/3")
    assert c.decode_batch(np.zeros((0, c.n_coded), np.float32)).shape == (0, c.k_info)
    bits, lf = c.decode_batch(np.zeros((0, c.n_coded), np.float32), return_lfinal=True)
    assert bits.shape == lf.shape == (0, c.k_info)
    with pytest.raises(IndexError):   # the row-length check still applies to an empty batch
        c.decode_batch(np.zeros((0, c.n_coded - 1), np.float32))
    LeA, LeB = M.bcjr_max_log_map_batch(*np.zeros((4, 0, 48), np.float32), *np.zeros((2, 0, 48)), *_tabs(), 48, 0.7)
    assert LeA.shape == LeB.shape == (0, 48)
    LeA, LeB = M.bcjr_max_log_map(*np.zeros((4, 0), np.float32), *np.zeros((2, 0)), *_tabs(), 0, 0.7)
    assert LeA.shape == LeB.shape == (0,) and LeA.dtype == np.float64
    dl = torch.zeros((0, c.n_coded), dtype=torch.float32, device="cuda")
    assert c.decode_device(dl).shape == (0, c.k_info)
    u8 = torch.zeros((0, c.k_info), dtype=torch.uint8, device="cuda")
    assert c.encode_device(u8).shape[0] == 0
    cons = D.constellation("16QAM")
    planes = torch.empty(16, dtype=torch.float32, device="cuda")
    c.demap_planes_device(torch.zeros((0, 1128), dtype=torch.complex64, device="cuda"), cons, 4, 0.1, planes)
    c.decode_planes_device(planes, 0, torch.empty((0, c.k_info), dtype=torch.int32, device="cuda"))
    assert D.compute_llr(np.zeros(0, np.complex64), "16QAM", 0.1).size == 0
    torch.cuda.synchronize()
    h = c.handle.h
    assert NT.lib().tdec_decode_batch(h, -1, None, c.n_coded, None, None) == -1
    assert NT.lib().tdec_siso_batch(h, -1, *[None] * 6, ctypes.c_double(0.7), None, None) == -1
    assert NT.lib().tdec_reserve(h, -1) == -1


@pytest.mark.parametrize("mod", ["BPSK", "QPSK", "8PSK", "16QAM", "64QAM", "256QAM"])
def test_demap_batch_fixed_signature(mod):
    """tdec_demap_batch (SURVEY §8(b) signature) = compute_llr with a Python-float
    noise_var, rounded to f32, in either sign convention."""
    from modulations_amd import _native as NT
    rng = np.random.default_rng(7)
    cons = D.constellation(mod)
    n = 3001
    syms = (cons[rng.integers(0, len(cons), n)] + 0.3 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)))
    syms = syms.astype(np.complex64)
    bps = D.MODULATIONS[mod]["bps"]
    mod_id = ("BPSK", "QPSK", "8PSK", "16QAM", "64QAM", "256QAM").index(mod)
    for sign in (1, -1):
        out = np.zeros(n * bps, np.float32)
        NT.check(NT.lib().tdec_demap_batch(0, mod_id, sign, NT.ptr(syms), n, 0.125, NT.ptr(out)))
        want = (sign * D.compute_llr(syms, mod, 0.125)).astype(np.float32)
        assert np.array_equal(out, want), (mod, sign)
        if sign == 1:   # and the oracle, on the same f32 table / dtype rules
            _, div32, nve = D.demap_mode(np.complex64, cons.dtype, 0.125)
            assert np.array_equal(out, O.demap(syms, cons, bps, nve, div_f32=div32).astype(np.float32))


def test_host_decode_in_chunks(monkeypatch):
    """tdec_decode_batch and tdec_siso_batch walk a large host batch in chunks
    (bounded device memory); a small TDEC_HOST_CHUNK forces several chunks and
    a ragged last one, results identical to the oracle."""
    monkeypatch.setenv("TDEC_HOST_CHUNK", "70")
    rng = np.random.default_rng(21)
    c = M.DVBRCS2_Turbo(48, "1/2")
    _, llr = _awgn_llrs(rng, c, 229, 1.5, 0.5)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    t, _ = O.trellis()
    rb, rl = O.decode_batch(llr, 48, c.punct["period"], T.puncture_matrix(c.punct), 8, c.perm, c.inv_perm, t,
                            want_lfinal=True)
    assert np.array_equal(bits, rb) and np.array_equal(lf, rl)
    n, B = 50, 151
    Lc = (rng.standard_normal((4, B, n)) * 4).astype(np.float32)
    La = rng.standard_normal((2, B, n)) * 9
    M._SISO_CACHE.clear()
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), n, 0.7)
    for b in (0, 69, 70, 139, 140, 150):
        rA, rB = O.siso(*Lc[:, b], *La[:, b], t, 0.7)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB), b


@pytest.mark.parametrize("n", [48, 212, 752, 37])
def test_state_per_lane_siso_prototype_bit_exact(monkeypatch, n):
    """The north star's mapping (one state per lane, tdec_spl.hip), kept as a
    timed A/B prototype: same SISO bits as the oracle."""
    monkeypatch.setenv("TDEC_SISO_SPL", "1")
    rng = np.random.default_rng(n)
    t, _ = O.trellis()
    B = 37
    Lc = (rng.standard_normal((4, B, n)) * 3).astype(np.float32)
    La = rng.standard_normal((2, B, n)) * 6
    LeA, LeB = M.bcjr_max_log_map_batch(*Lc, *La, *_tabs(), n, 0.7)
    for b in (0, 17, B - 1):
        rA, rB = O.siso(Lc[0, b], Lc[1, b], Lc[2, b], Lc[3, b], La[0, b], La[1, b], t, 0.7)
        assert np.array_equal(LeA[b], rA) and np.array_equal(LeB[b], rB), b


def test_reference_test_py_recipe_through_the_drop_in():
    """The reference's test.py recipe (QPSK r=1/2 N=752 8 iterations, its
    -(2 sqrt 2)/N0 LLR scale) through DVBRCS2_Turbo exactly as test.py calls it
    (codec.decode(llrs) per frame) and as a batch: the reference's bits."""
    from conftest import golden
    g = golden("testpy")
    c = M.DVBRCS2_Turbo(752, "1/2", 8, inv_perm="numpy-avx512")
    assert np.array_equal(c.inv_perm, g["inv_perm"])
    llrs = np.stack([g[f"llr_{i}"] for i in range(9)])
    want = np.stack([g[f"bits_{i}"] for i in range(9)])
    assert np.array_equal(c.decode_batch(llrs), want)
    for i in (0, 8):
        assert np.array_equal(c.decode(g[f"llr_{i}"]), g[f"bits_{i}"])
