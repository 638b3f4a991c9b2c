"""GPU parity of the modem front-end: libmodem.so through
its C ABI (modulations_amd.modem) against the reference's golden vectors and
the C oracle.  Bit-exact for mappers, hard decisions and the IQ format (8PSK on
complex64: exact away from a 1e-5 band around the sector boundaries, see
test_modem_host.psk8_boundary_ok); the FIR forms within 1e-13 of the output
scale (the reference's BLAS / scipy summation order is not defined)."""
import os
import warnings

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import modem as MM  # noqa: E402
from test_modem_host import MO_MODS, QAM, SDR_MODS, psk8_boundary_ok, sdr_demod_oracle  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def G():
    return np.load(os.path.join(ROOT, "tests", "golden", "modem.npz"), allow_pickle=False)


def close(y, ref, tol=1e-13):
    assert y.shape == ref.shape and y.dtype == ref.dtype
    scale = max(np.max(np.abs(ref)), 1e-300) if ref.size else 1.0
    assert (np.max(np.abs(y - ref)) if ref.size else 0.0) <= tol * scale


# ---------------------------------------------------------------- mappers --------------------
@pytest.mark.parametrize("mod,bps", SDR_MODS)
def test_sdr_modulate_golden(G, mod, bps):
    m = MM.SDRModem()
    sy = m.modulate(G[f"sdr_bits_{mod}"], mod)
    ref = G[f"sdr_mod_{mod}"]
    assert sy.dtype == ref.dtype and np.array_equal(sy, ref)


@pytest.mark.parametrize("mod", ["BPSK", "QPSK", "8PSK", "16QAM"])
def test_harness_mappers_golden(G, mod):
    sy = MM.MODULATIONS[mod]["mod"](G[f"h_bits_{mod}"])
    ref = G[f"h_mod_{mod}"]
    assert sy.dtype == ref.dtype and np.array_equal(sy, ref)


@pytest.mark.parametrize("name,bps", MO_MODS)
def test_modulator_mappers_golden(G, name, bps):
    mo = MM.Modulator()
    sy = getattr(mo, f"mod_{name}")(G[f"mo_bits_{name}"])
    ref = G[f"mo_mod_{name}"]
    assert sy.dtype == ref.dtype and np.array_equal(sy, ref)


def test_mapper_random_vs_oracle_and_edges():
    rng = np.random.default_rng(3)
    for mod, bps in SDR_MODS:
        t = D.constellation(mod)
        for n in (1, bps - 1, 12345, 250_001):
            if n <= 0:
                continue
            bits = rng.integers(0, 2, n).astype(np.uint8)
            assert np.array_equal(MM.map_bits(bits, bps, t), O.modem_map(bits, bps, t)), (mod, n)
        assert MM.map_bits(np.zeros(0, np.uint8), bps, t).shape == (0,)
    with pytest.raises(ValueError):
        MM.qpsk_mod([0, 1, 3])


# ---------------------------------------------------------------- hard demods ----------------
@pytest.mark.parametrize("mod,bps", SDR_MODS)
def test_sdr_demodulate_golden(G, mod, bps):
    m = MM.SDRModem()
    for key in ("sdr_rx_", "sdr_rx128_"):
        rx = G[key + mod]
        got = m.demodulate(rx, mod)
        ref = G[key.replace("rx", "demod") + mod]
        assert got.dtype == ref.dtype
        if mod == "8PSK" and rx.dtype == np.complex64:
            assert psk8_boundary_ok(rx, got, ref) <= 4
        else:
            assert np.array_equal(got, ref), key
    e = m.demodulate(np.zeros(0, np.complex64), mod)
    assert e.dtype == G[f"sdr_emptydemod_{mod}"].dtype and e.size == 0
    if str(G[f"sdr_nanerr_{mod}"]) == "ValueError":
        with pytest.raises(ValueError):
            m.demodulate(np.array([1 + 1j, np.nan + 0j], np.complex64), mod)
    else:
        m.demodulate(np.array([np.nan + 0j], np.complex64), mod)


@pytest.mark.parametrize("mod", ["BPSK", "QPSK", "8PSK", "16QAM"])
def test_harness_demods_golden(G, mod):
    rx = G[f"sdr_rx_{mod}"]
    got = MM.MODULATIONS[mod]["demod"](rx)
    if mod == "8PSK":
        assert psk8_boundary_ok(rx, got, G[f"h_demod_{mod}"]) <= 4
    else:
        assert np.array_equal(got, G[f"h_demod_{mod}"])


@pytest.mark.parametrize("name,bps", MO_MODS)
def test_modulator_demods_golden(G, name, bps):
    mo = MM.Modulator()
    f = getattr(mo, f"demod_{name}")
    for key in ("mo_demod_", "mo_demod128_", "mo_nandemod_"):
        rx = G["mo_nanrx_" + name] if key == "mo_nandemod_" else G["mo_rx_" + name]
        if key == "mo_demod128_":
            rx = rx.astype(np.complex128)
        got = f(rx)
        ref = G[key + name]
        assert got.dtype == ref.dtype
        if name == "8psk" and key == "mo_demod_":
            assert psk8_boundary_ok(rx, got, ref) <= 8
        else:
            assert np.array_equal(got, ref), key


def test_demods_random_vs_oracle():
    """Large noisy inputs, complex64 and complex128, every rule vs the oracle."""
    rng = np.random.default_rng(11)
    mo = MM.Modulator()
    for mod, bps in SDR_MODS:
        t = D.constellation(mod)
        for dt in (np.complex64, np.complex128):
            n = 200_003
            rx = (t[rng.integers(0, len(t), n)] + 0.2 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)))
            rx = rx.astype(dt)
            got = MM.SDRModem().demodulate(rx, mod)
            ref = sdr_demod_oracle(rx, mod)
            if mod == "8PSK" and dt == np.complex64:
                assert psk8_boundary_ok(rx, got, ref) <= 3
            else:
                assert np.array_equal(got, ref), (mod, dt)
    for M in (16, 64):
        c = mo._qam_const(M)[0]
        rx = (c[rng.integers(0, M, 100_000)] + 0.15 * (rng.standard_normal(100_000) + 1j *
                                                       rng.standard_normal(100_000))).astype(np.complex64)
        got = mo._demod_qam_generic(rx, M)
        ref = O.modem_demod(rx, 4, int(np.log2(M)), cons=c)[0]
        assert np.array_equal(got, ref), M


def test_noise_free_round_trip_full_size():
    """map -> demod is the identity on noise-free symbols (1M symbols per rule)."""
    rng = np.random.default_rng(5)
    m = MM.SDRModem()
    for mod, bps in SDR_MODS:
        bits = rng.integers(0, 2, 1_000_000 * bps).astype(np.uint8)
        assert np.array_equal(m.demodulate(m.modulate(bits, mod), mod), bits), mod
    mo = MM.Modulator()
    for name, bps in MO_MODS:
        bits = rng.integers(0, 2, 300_000 * bps).astype(np.uint8)
        sy = getattr(mo, f"mod_{name}")(bits)
        assert np.array_equal(getattr(mo, f"demod_{name}")(sy), bits), name


# ---------------------------------------------------------------- pulse shaping ---------------
def test_upsample_filter_golden(G):
    m = MM.SDRModem()
    for n in (500, 20, 7):
        close(m._upsample_filter(G[f"sdr_upin_{n}"]), G[f"sdr_upout_{n}"])
    close(MM.upsample_filter(G["h_upin"], 8, G["sdr_taps_8"]), G["h_upout"])
    with pytest.raises(ValueError):
        m._upsample_filter(np.zeros(0, np.complex64))


def test_modulator_filters_golden(G):
    mo = MM.Modulator()
    close(mo.apply_pulse_shaping(G["mo_shape_in"]), G["mo_shaped"])
    close(mo.matched_filter(G["mo_mf_in"]), G["mo_mf_out"])
    close(mo.matched_filter(G["mo_mf64_in"]), G["mo_mf64_out"])
    close(mo.matched_filter(G["mo_mf_in"][:10]), G["mo_mf_short_out"])
    close(mo.matched_filter(G["mo_mf_real_in"]), G["mo_mf_real_out"])
    e = mo.matched_filter(np.ones(3, np.complex64)[:0])
    assert e.dtype == np.complex64 and e.size == 0


def test_fir_random_vs_oracle():
    rng = np.random.default_rng(8)
    for up, down, L, n, dt in ((4, 1, 101, 30_000, np.complex64), (8, 1, 49, 5_000, np.complex128),
                               (1, 8, 49, 80_000, np.complex128), (1, 4, 101, 60_000, np.complex64),
                               (3, 2, 17, 7_777, np.complex64), (16, 1, 255, 2_000, np.complex64)):
        x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(dt)
        h = rng.standard_normal(L)
        n_full = (n - 1) * up + L
        for off in (0, (L - 1) // 2, L - 1):
            n_out = (n_full - off + down - 1) // down
            close(MM.fir(x, h, up, down, off, n_out), O.modem_fir(x, h, up, down, off, n_out), 1e-12)


# ---------------------------------------------------------------- IQ format ------------------
def test_iq_golden(G, tmp_path):
    m = MM.SDRModem()
    for k in ("128", "64", "tiny", "nan", "inf"):
        f = str(tmp_path / f"s{k}.iq")
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            m._save_iq(G["iq_sig" + k], f)
        assert np.array_equal(np.fromfile(f, np.int8), G["iq_saved" + k]), k
    f = str(tmp_path / "r.iq")
    G["iq_raw"].tofile(f)
    d = m._load_iq(f)
    assert d.dtype == np.complex64 and np.array_equal(d, G["iq_loaded"])
    assert np.array_equal(MM.load_iq(f), G["iq_loaded_h"])
    with pytest.raises(ValueError):
        m._save_iq(np.zeros(0, np.complex128), f)


def test_iq_odd_lengths_like_numpy():
    raw = np.array([3, 200, 77, 9, 14], np.uint8)
    for n in (1, 3):
        I = (raw[:n][0::2].astype(np.float32) - 127.5) / 127.5
        Q = (raw[:n][1::2].astype(np.float32) - 127.5) / 127.5
        assert np.array_equal(MM.iq_dequantize(raw[:n]), I + 1j * Q)
    with pytest.raises(ValueError):
        MM.iq_dequantize(raw)


def test_iq_random_vs_oracle_full_size():
    rng = np.random.default_rng(9)
    for dt in (np.complex64, np.complex128):
        sig = (rng.standard_normal(3_000_000) + 1j * rng.standard_normal(3_000_000)).astype(dt)
        assert np.array_equal(MM.iq_quantize(sig), O.modem_iq_quantize(sig)), dt
    raw = rng.integers(0, 256, 4_000_000).astype(np.uint8)
    assert np.array_equal(MM.iq_dequantize(raw), O.modem_iq_dequantize(raw))


# ---------------------------------------------------------------- device-resident API ----------
def test_device_api_matches_host_api():
    rng = np.random.default_rng(12)
    dev = torch.device("cuda:0")
    t = D.constellation("16QAM")
    bits = rng.integers(0, 2, 4 * 100_001).astype(np.uint8)
    sy = MM.map_device(torch.from_numpy(bits).to(dev), 4, t)
    assert np.array_equal(sy.cpu().numpy(), MM.map_bits(bits, 4, t))
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    b = MM.demod_device(sy, MM.QAM_AXIS, 4, labels=MM._INV[2], scale=np.sqrt(10), nan_count=cnt)
    assert np.array_equal(b.cpu().numpy(), bits) and int(cnt.item()) == 0
    taps = MM.rrc_taps(4)
    y = MM.fir_device(sy, taps, 4, 1, 50, sy.numel() * 4)
    assert np.allclose(y.cpu().numpy(), MM.fir(sy.cpu().numpy(), taps, 4, 1, 50, sy.numel() * 4), rtol=0,
                       atol=1e-13)
    iq = MM.iq_quantize_device(y)
    assert np.array_equal(iq.cpu().numpy(), MM.iq_quantize(y.cpu().numpy()))
    back = MM.iq_dequantize_device(iq.view(torch.uint8))
    assert np.array_equal(back.cpu().numpy(), MM.iq_dequantize(iq.cpu().numpy().view(np.uint8)))
    nan_syms = torch.tensor([1 + 1j, float("nan") + 0j], dtype=torch.complex64, device=dev)
    cnt.zero_()
    MM.demod_device(nan_syms, MM.PSK8, 3, labels=MM._INV[3], nan_count=cnt)
    assert int(cnt.item()) == 1
