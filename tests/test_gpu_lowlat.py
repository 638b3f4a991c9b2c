"""The low-latency (state-per-lane) max-log decoder, tdec_lowlat.hip: small
batches of DVBRCS2_Turbo.decode / decode_batch / decode_device run 16 lanes per
codeword where the frame decoder does not (N > 805, or TDEC_FRAME=0, which this
module sets so that it tests this decoder; tests/test_gpu_frame.py covers the frame
decoder).  Every case is compared bit for bit
(hard bits and L_final, IEEE ==) with the C oracle, the restatement of
dvb_rcs2_turbo.py:464-537 pinned to the reference's golden vectors."""
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


@pytest.fixture(autouse=True)
def _lowlat_decoder():
    import os
    old = os.environ.get("TDEC_FRAME")
    os.environ["TDEC_FRAME"] = "0"   # read per call by the library
    yield
    if old is None:
        os.environ.pop("TDEC_FRAME", None)
    else:
        os.environ["TDEC_FRAME"] = old


def _llrs(rng, c, B, scale, noise):
    info = rng.integers(0, 2, (B, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * scale for b in info]).astype(np.float32)
    llr += (rng.standard_normal(llr.shape) * noise).astype(np.float32)
    return llr


def _oracle(c, llr):
    t, _ = O.trellis()
    return O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm, c.inv_perm,
                          t, want_lfinal=True, nthreads=8)


@pytest.mark.parametrize("n,rate", [(752, "1/2"), (752, "1/3"), (212, "1/3"), (48, "1/3"), (220, "2/3"),
                                    (848, "1/2"), (64, "3/4")])
@pytest.mark.parametrize("B", [1, 3, 4, 5, 67])
def test_lowlat_decode_matches_oracle(n, rate, B):
    rng = np.random.default_rng(1000 * n + B)
    c = M.DVBRCS2_Turbo(n, rate)
    llr = _llrs(rng, c, B, 2.0, 1.6)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = _oracle(c, llr)
    assert np.array_equal(bits, rb) and np.array_equal(lf, rl)


def test_lowlat_single_decode_and_extreme_inputs():
    c = M.DVBRCS2_Turbo(752, "1/2")
    rng = np.random.default_rng(5)
    cases = [np.zeros(c.n_coded, np.float32),                                # all-zero: ties everywhere
             (rng.standard_normal(c.n_coded) * 1e4).astype(np.float32),      # extrinsics clip at +-300
             (rng.standard_normal(c.n_coded) * 1e-3).astype(np.float32),
             _llrs(rng, c, 1, 20.0, 0.0)[0]]                                  # noise-free
    for llr in cases:
        rb, rl = _oracle(c, llr[None])
        bits = c.decode(llr)
        assert np.array_equal(bits, rb[0])
        b2, l2 = c.decode_batch(llr[None], return_lfinal=True)
        assert np.array_equal(l2, rl)


def test_lowlat_device_api_and_iterations():
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(9)
    for it in (1, 2, 5):
        c = M.DVBRCS2_Turbo(212, "1/3", it)
        llr = _llrs(rng, c, 37, 2.0, 1.8)
        c.reserve(37)
        bits = torch.empty((37, c.k_info), dtype=torch.int32, device=dev)
        c.decode_device(torch.from_numpy(llr).to(dev), bits)
        torch.cuda.synchronize()
        rb, _ = _oracle(c, llr)
        assert np.array_equal(bits.cpu().numpy(), rb)


@pytest.mark.parametrize("n,rate", [(752, "1/3"), (212, "1/3"), (48, "1/3"), (220, "2/3"), (64, "3/4")])
def test_throughput_decoder_at_small_batches(n, rate):
    """A handle reserved for a large batch keeps the one-codeword-per-lane decoder
    for small ones (no low-latency workspace): that kernel against the oracle at
    ragged tile counts."""
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(77 + n)
    c = M.DVBRCS2_Turbo(n, rate)
    c.reserve(70_000)
    for B in (1, 5, 67):
        llr = _llrs(rng, c, B, 2.0, 1.6)
        bits = torch.empty((B, c.k_info), dtype=torch.int32, device=dev)
        lf = torch.empty((B, c.k_info), dtype=torch.float64, device=dev)
        planes = torch.empty(c.planes_bytes(B) // 4, dtype=torch.float32, device=dev)
        c.depuncture_device(torch.from_numpy(llr).to(dev), planes)
        c.decode_planes_device(planes, B, bits, lf)       # no reserve(B): the 70 000 workspace
        torch.cuda.synchronize()
        rb, rl = _oracle(c, llr)
        assert np.array_equal(bits.cpu().numpy(), rb) and np.array_equal(lf.cpu().numpy(), rl)


@pytest.mark.parametrize("n,rate,interleaver", [(212, "1/3", "reference"), (752, "1/2", "valid-perm")])
def test_lowlat_large_batch_matches_oracle(n, rate, interleaver):
    """B above the 2 048 resident waves (below the small-batch limit, 8 192 / 12 288
    for the frame decoder, 4 096 for the state-per-lane one): more than one round of
    small-batch blocks; with a true permutation every position is in
    perm's image, so decoder 1 computes every extrinsic (the used-position list
    is the identity)."""
    rng = np.random.default_rng(77 + n)
    c = M.DVBRCS2_Turbo(n, rate, interleaver=interleaver)
    B = 2500 if n == 212 else 300
    llr = _llrs(rng, c, B, 2.0, 1.6)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    rb, rl = _oracle(c, llr)
    assert np.array_equal(bits, rb) and np.array_equal(lf, rl)


def test_reserve_small_batch_on_a_block_too_long_for_the_small_batch_decoders():
    """C ABI only (the Python codec restricts N to the standard table): N = 6 000
    couples, beyond both the frame decoder's LDS (N <= 805) and the state-per-lane
    decoder's 64 KiB tables (N <= 5 461).  tdec_reserve of a small batch must
    reserve the throughput decoder's workspace, and the decode runs there, equal
    to the oracle (one predicate for reserve and decode)."""
    import ctypes as C
    from modulations_amd import _native
    L = _native.lib()
    n, B = 6000, 3
    perm = ((np.arange(n, dtype=np.int64) * 7 + 3) % n).astype(np.int32)   # a true permutation
    inv = np.argsort(perm, kind="stable").astype(np.int32)
    c = M.DVBRCS2_Turbo(48, "1/3")
    tabs = T.packed_tables(c.next_state, c.out_W, c.out_Y, c.prev_state, c.prev_input)
    pm = T.puncture_matrix(c.punct)
    h = C.c_void_p()
    assert L.tdec_create(0, n, c.punct["period"], pm.ctypes.data, 8, 0, perm.ctypes.data, inv.ctypes.data,
                         tabs.ctypes.data, C.byref(h)) == 0, L.tdec_last_error()
    try:
        assert L.tdec_reserve(h, B) == 0, L.tdec_last_error()
        rng = np.random.default_rng(6000)
        n_coded = 6 * n   # rate 1/3: A, B, W1, Y1, W2, Y2 per couple
        llr = (rng.standard_normal((B, n_coded)) * 2).astype(np.float32)
        bits = np.zeros((B, 2 * n), np.int32)
        lf = np.zeros((B, 2 * n), np.float64)
        assert L.tdec_decode_batch(h, B, llr.ctypes.data, n_coded, bits.ctypes.data, lf.ctypes.data) == 0, \
            L.tdec_last_error()
    finally:
        L.tdec_destroy(h)
    t, _ = O.trellis()
    rb, rl = O.decode_batch(llr, n, c.punct["period"], pm, 8, perm, inv, t, want_lfinal=True, nthreads=8)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)
