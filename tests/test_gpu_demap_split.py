"""The split demapper (TDEC_DM_SPLIT, csrc/tdec_kernels.hip): k_demap_planes runs
only the fast exact search for square 16 / 64 / 256QAM and lists the symbols it
declines; k_demap_fix gives those the full chain and rewrites their plane
entries, and redoes every symbol of a tile whose declines overflowed the list.

Checked against the host chain the reference runs (compute_llr,
test_sdr_with_coding.py:200-225, decoder sign, truncated / zero-padded as
:474-478 to the decoder's LLR count), put into the same tile planes by the depuncture kernel:
the planes must be equal (NaN == NaN), on symbols that are declined often
(ties, near-ties, NaN / inf, out-of-grid) and on a batch whose declines
overflow the list (most symbols NaN)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _adversarial(cons, rng, shape):
    """Noisy points mixed with exact points, bisector ties, near-ties, far / tiny /
    huge values and NaN / inf, shuffled over the batch."""
    n = int(np.prod(shape))
    lv = np.unique(cons.real.astype(np.float64))
    mids = (lv[:-1] + lv[1:]) / 2
    k = n // 10
    parts = [cons[rng.integers(0, len(cons), n - 7 * k)] + 0.2 * (rng.standard_normal(n - 7 * k) +
                                                                 1j * rng.standard_normal(n - 7 * k)),
             cons[rng.integers(0, len(cons), k)],
             rng.choice(mids, k) + 1j * rng.choice(lv, k),
             rng.choice(mids, k) + 1j * rng.choice(mids, k),
             np.nextafter(rng.choice(mids, k), 9) + 1j * np.nextafter(rng.choice(mids, k), -9),
             10 * (rng.standard_normal(k) + 1j * rng.standard_normal(k)),
             1e-20 * (rng.standard_normal(k) + 1j * rng.standard_normal(k)),
             rng.choice(np.array([np.nan, np.inf, -np.inf + 1j, 1 + np.nan * 1j, 3e38 + 3e38j]), k)]
    s = np.concatenate(parts)
    rng.shuffle(s)
    return s.reshape(shape).astype(np.complex64)


def _check(c, syms, mod, nv, cons=None):
    cons = D.constellation(mod) if cons is None else cons
    bps = D.MODULATIONS[mod]["bps"]
    B = syms.shape[0]
    nv = nv if isinstance(nv, (np.floating,)) else np.float64(nv)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, nv)
    c.reserve(B)
    planes = torch.empty(c.planes_bytes(B) // 4, dtype=torch.float32, device="cuda")
    c.demap_planes_device(torch.from_numpy(syms).cuda(), cons, bps, nve, planes, div_f32=div32)
    # the host chain on the distinct finite rows only (NaN symbols give NaN LLRs)
    flat = syms.reshape(-1)
    llr = np.full(flat.size * bps, np.nan, np.float64)
    fin = ~np.isnan(flat)
    llr.reshape(-1, bps)[fin] = (-O.demap(flat[fin], cons, bps, nve, div_f32=div32)).reshape(-1, bps)
    llr = llr.reshape(B, -1)
    # zero-padded / truncated to the decoder's LLR count, the de-puncture walk
    # (include/tdec.h, tdec_demap_planes_dev).  It equals the reference's n_coded
    # when the puncture period divides N; otherwise (N = 212 / 752 at rate 2/3)
    # n_coded is shorter than the walk and the reference's chain raises IndexError
    # in decode() (test_sdr_with_coding.py:474-480, dvb_rcs2_turbo.py:476-487)
    L = c.handle.llr_len
    ref_llr = np.zeros((B, L), np.float32)
    m = min(L, llr.shape[1])
    ref_llr[:, :m] = llr[:, :m]
    ref = torch.empty_like(planes)
    c.depuncture_device(torch.from_numpy(ref_llr).cuda(), ref)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(planes.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("mod,n,rate", [("16QAM", 752, "1/3"), ("64QAM", 212, "1/2"), ("256QAM", 752, "1/3"),
                                        ("256QAM", 48, "3/4"), ("16QAM", 212, "2/3"), ("64QAM", 752, "2/3")])
def test_split_planes_equal_host_chain(mod, n, rate):
    rng = np.random.default_rng(sum(map(ord, mod)) + n)
    c = M.DVBRCS2_Turbo(n, rate)
    bps = D.MODULATIONS[mod]["bps"]
    S = -(-c.n_coded // bps)
    _check(c, _adversarial(D.constellation(mod), rng, (130, S)), mod, 0.04)


@pytest.mark.parametrize("mod,n,rate", [("BPSK", 752, "1/3"), ("BPSK", 48, "3/4"), ("QPSK", 212, "1/3"),
                                        ("QPSK", 752, "2/3"), ("8PSK", 752, "1/2"), ("8PSK", 752, "3/4"),
                                        ("8PSK", 64, "2/3")])
def test_inline_planes_equal_host_chain(mod, n, rate):
    """The tables demapped inline (no split) through the same plane kernel and its
    planar LDS tile (column b * ns + symbol): BPSK's 96-symbol items (more
    symbols than lanes), 8PSK's straddling symbols at 3/4 (2068 LLRs, 3 per
    symbol), a ragged last tile (130 codewords), adversarial symbols."""
    rng = np.random.default_rng(sum(map(ord, mod)) + n + len(rate))
    c = M.DVBRCS2_Turbo(n, rate)
    bps = D.MODULATIONS[mod]["bps"]
    S = -(-c.n_coded // bps)
    _check(c, _adversarial(D.constellation(mod), rng, (130, S)), mod, 0.04)


def test_split_overflowing_declines_redo_their_tiles():
    """64QAM, 8 192 codewords x 752 symbols with 90 % NaN: 5.5 M declines against
    a list of 2 M entries, so tiles overflow and are redone whole."""
    rng = np.random.default_rng(77)
    mod = "64QAM"
    c = M.DVBRCS2_Turbo(752, "1/3")
    cons = D.constellation(mod)
    B, S = 8192, -(-c.n_coded // 6)
    syms = (cons[rng.integers(0, 64, (B, S))] + 0.1 * (rng.standard_normal((B, S)) +
                                                        1j * rng.standard_normal((B, S)))).astype(np.complex64)
    syms[rng.random((B, S)) < 0.9] = np.nan
    _check(c, syms, mod, 0.02)


@pytest.mark.parametrize("kind", ["ring16", "natural64"])
def test_tables_the_fast_search_cannot_take_stay_inline(kind):
    """A 16-point two-ring table (not separable) and a 64QAM grid labelled in natural
    binary order (separable, not Gray): the split path would decline every symbol,
    so these run the inline chain; the planes still equal the host chain."""
    rng = np.random.default_rng(5 if kind == "ring16" else 6)
    if kind == "ring16":
        cons = np.concatenate([np.exp(1j * (np.pi / 4 * np.arange(4) + np.pi / 4)),
                               2.6 * np.exp(1j * (np.pi / 6 * np.arange(12)))]).astype(np.complex64)
        bps = 4
    else:
        lv = np.arange(-7, 8, 2, dtype=np.float64) / np.sqrt(42)
        cons = (lv[np.arange(64) >> 3] + 1j * lv[np.arange(64) & 7]).astype(np.complex64)
        bps = 6
    c = M.DVBRCS2_Turbo(212, "1/3")
    B, S = 70, -(-c.n_coded // bps)
    syms = (cons[rng.integers(0, len(cons), (B, S))] + 0.2 * (rng.standard_normal((B, S)) +
                                                              1j * rng.standard_normal((B, S)))).astype(np.complex64)
    syms[0, :5] = np.nan
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(0.05))
    c.reserve(B)
    planes = torch.empty(c.planes_bytes(B) // 4, dtype=torch.float32, device="cuda")
    c.demap_planes_device(torch.from_numpy(syms).cuda(), cons, bps, nve, planes, div_f32=div32)
    llr = np.stack([-O.demap(r, cons, bps, nve, div_f32=div32) for r in syms])
    # zero-padded / truncated to the decoder's LLR count, the de-puncture walk
    # (include/tdec.h, tdec_demap_planes_dev).  It equals the reference's n_coded
    # when the puncture period divides N; otherwise (N = 212 / 752 at rate 2/3)
    # n_coded is shorter than the walk and the reference's chain raises IndexError
    # in decode() (test_sdr_with_coding.py:474-480, dvb_rcs2_turbo.py:476-487)
    L = c.handle.llr_len
    ref_llr = np.zeros((B, L), np.float32)
    m = min(L, llr.shape[1])
    ref_llr[:, :m] = llr[:, :m]
    ref = torch.empty_like(planes)
    c.depuncture_device(torch.from_numpy(ref_llr).cuda(), ref)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(planes.cpu().numpy(), ref.cpu().numpy())


@pytest.mark.parametrize("case", ["f32_division", "f64_table", "nv_outside_fast_range", "nv_floor"])
def test_split_16qam_arithmetic_variants(case):
    """16QAM's closed-form search and unscaled divisions (TDEC_DM_PAIRS,
    TDEC_DM_FAST64) on every arithmetic the reference's dtypes select: the f32
    quotient (float32 noise variance, numpy's weak scalar rule), a complex128
    table (f64 throughout), a noise variance outside the unscaled division's
    range (the streamed search and the compiler's division run) and the 0.005
    floor."""
    rng = np.random.default_rng(sum(map(ord, case)))
    mod = "16QAM"
    c = M.DVBRCS2_Turbo(212, "1/2")
    S = -(-c.n_coded // 4)
    cons = D.constellation(mod)
    nv = {"f32_division": np.float32(0.037), "f64_table": 0.037, "nv_outside_fast_range": 1e5,
          "nv_floor": 1e-4}[case]
    if case == "f64_table":
        cons = cons.astype(np.complex128)
    syms = _adversarial(cons, rng, (70, S))
    if case == "nv_outside_fast_range":
        syms = (syms * 300).astype(np.complex64)
    _check(c, syms, mod, nv, cons)


@pytest.mark.parametrize("mod", ["64QAM", "256QAM"])
@pytest.mark.parametrize("case", ["f32_division", "f64_table", "nv_outside_fast_range"])
def test_split_gray_arithmetic_variants(mod, case):
    """The Gray search's pre-checked unscaled sequences (TDEC_DM_GRAYPRE) on the
    f32 quotient, a complex128 table, and a noise variance outside their range
    (every symbol then declines to the full chain)."""
    rng = np.random.default_rng(sum(map(ord, mod + case)))
    c = M.DVBRCS2_Turbo(212, "1/2")
    bps = D.MODULATIONS[mod]["bps"]
    S = -(-c.n_coded // bps)
    cons = D.constellation(mod)
    nv = {"f32_division": np.float32(0.021), "f64_table": 0.021, "nv_outside_fast_range": 1e5}[case]
    if case == "f64_table":
        cons = cons.astype(np.complex128)
    syms = _adversarial(cons, rng, (66, S))
    _check(c, syms, mod, nv, cons)
