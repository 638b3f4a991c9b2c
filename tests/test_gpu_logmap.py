"""log-MAP (BASELINE configs[3]) end to end on the GPU.

* configs[3]'s chain: Gray 8PSK (sdr_modem.py:120-130) over AWGN, the fused
  soft demap + de-puncture (3008 coded bits -> 1003 symbols, one zero pad bit,
  truncated back as test_sdr_with_coding.py:474-478), then the log-MAP turbo
  decoder at N=752 couples, r=1/2 -- bit for bit against the C oracle
  (algo=1: the build-defined max*, restated identically on both sides);
* the persistent tile loop of k_turbo_decode_logmap wrapping (a batch larger
  than resident waves x 64 codewords) at full size: determinism, shard
  equivalence, and oracle spot checks on the first / middle / last codewords.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("trans_tables")]

from oracle import oracle as O  # noqa: E402
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402
from modulations_amd.workload import DevicePipeline, make_symbols  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _oracle(codec, llr, algo=1, want_lfinal=False):
    t, _ = O.trellis()
    return O.decode_batch(llr, codec.N, codec.punct["period"], T.puncture_matrix(codec.punct), codec.iterations,
                          codec.perm, codec.inv_perm, t, algo=algo, nthreads=16, want_lfinal=want_lfinal)


def _rows(B, n_first, n_spread):
    """The first n_first rows and n_spread spread over the rest, the last included."""
    idx = np.unique(np.concatenate([np.arange(min(B, n_first)),
                                    np.linspace(min(B, n_first), B - 1, n_spread).astype(np.int64)]))
    assert idx[-1] == B - 1
    return idx


def _host_llrs(codec, syms_rows, mod, n0):
    cons = D.constellation(mod)
    bps = D.MODULATIONS[mod]["bps"]
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    return np.stack([-O.demap(r, cons, bps, nve, div_f32=div32)[:codec.n_coded] for r in syms_rows]).astype(np.float32)


@pytest.mark.parametrize("B", [96, 7232])
def test_8psk_demap_planes_to_logmap_decode_n752_r12(B):
    """B = 96: the frame decoder (small batches); B = 7 232 > LM_FRAME_MAX (7 168):
    the timed throughput kernel k_turbo_decode_logmap."""
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    assert codec.n_coded == 3008
    info, syms, n0 = make_symbols(codec, B, "8PSK", 3.0, 11, dev)
    assert syms.shape == (B, 1003)                        # 3008 bits + 1 zero pad bit -> 1003 symbols
    pipe = DevicePipeline(codec, "8PSK", B, dev)
    bits = pipe.run(syms, n0).clone()
    torch.cuda.synchronize()
    idx = _rows(B, 256, 256) if B > 96 else np.arange(B)
    llr = _host_llrs(codec, syms[torch.as_tensor(idx, device=dev)].cpu().numpy(), "8PSK", n0)
    assert np.array_equal(bits[torch.as_tensor(idx, device=dev)].cpu().numpy(), _oracle(codec, llr))
    # and through the LLR-row boundary (host demap -> f32 -> decode): the same bits
    if B == 96:
        assert np.array_equal(codec.decode_batch(llr), bits.cpu().numpy())


def test_logmap_full_size_tile_wrap():
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    B = 140_000                  # > 2048 resident waves x 64 codewords on MI355X: the persistent loop wraps
    info, syms, n0 = make_symbols(codec, B, "8PSK", 3.0, 5, dev)
    pipe = DevicePipeline(codec, "8PSK", B, dev)
    b1 = pipe.run(syms, n0).clone()
    b2 = pipe.run(syms, n0).clone()
    torch.cuda.synchronize()
    assert torch.equal(b1, b2)                            # deterministic
    h = B // 3 + 5                                        # shard equivalence: two launches == one
    pa = DevicePipeline(codec, "8PSK", h, dev)
    pb = DevicePipeline(codec, "8PSK", B - h, dev)
    ba = pa.run(syms[:h].contiguous(), n0).clone()
    bb = pb.run(syms[h:].contiguous(), n0).clone()
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([ba, bb]), b1)
    idx = [0, 1, 63, 64, 131_071, 131_072, B // 2, B - 65, B - 1]
    llr = _host_llrs(codec, syms[idx].cpu().numpy(), "8PSK", n0)
    assert np.array_equal(b1[idx].cpu().numpy(), _oracle(codec, llr))


def test_logmap_timed_kernel_vs_oracle_4096_rows():
    """The timed kernel itself (k_turbo_decode_logmap, configs[3]'s shape) against
    the oracle on 4 096 rows of a 140 000-codeword batch: the
    first 2 048 (32 tiles of the first round) and 2 048 spread over the batch, the
    ragged last tile and rows of every round of the persistent loop included; bits
    AND L_final, IEEE ==.  (~30 s of 16-thread oracle time.)"""
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    B = 140_000
    info, syms, n0 = make_symbols(codec, B, "8PSK", 3.0, 5, dev)
    pipe = DevicePipeline(codec, "8PSK", B, dev)
    b1 = pipe.run(syms, n0).clone()
    lf = torch.empty((B, codec.k_info), dtype=torch.float64, device=dev)
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=dev)
    codec.decode_planes_device(pipe.planes, B, bits, lfinal=lf)
    torch.cuda.synchronize()
    assert torch.equal(bits, b1)
    idx = _rows(B, 2048, 2048)
    assert len(idx) >= 4096
    ti = torch.as_tensor(idx, device=dev)
    llr = _host_llrs(codec, syms[ti].cpu().numpy(), "8PSK", n0)
    rb, rl = _oracle(codec, llr, want_lfinal=True)
    assert np.array_equal(bits[ti].cpu().numpy(), rb)
    np.testing.assert_array_equal(lf[ti].cpu().numpy(), rl)


# ---- the hardware primitives of the build-defined log-MAP -------------
def test_trans_tables_are_faithful(trans_tables):
    """v_exp_f32 / v_log_f32 on the grids the log-MAP feeds them: every output
    within 1 ulp of the correctly rounded value (exp2 / log2 in f64, rounded
    once).  These tables are what the oracle uses in the GPU session."""
    et, elo, lt, llo = trans_tables
    t = np.arange(elo, elo + et.size, dtype=np.uint64).astype(np.uint32).view(np.float32)
    cr = np.exp2(-t.astype(np.float64)).astype(np.float32)
    d = et.view(np.int32).astype(np.int64) - cr.view(np.int32).astype(np.int64)
    assert np.all(np.abs(d) <= 1) and np.all(np.isfinite(et))
    e_off = np.mean(d != 0)
    w = np.arange(llo, llo + lt.size, dtype=np.uint64).astype(np.uint32).view(np.float32)
    cr = np.log2(w.astype(np.float64)).astype(np.float32)
    # log2 near 1 is tiny: compare in ulps of the result
    d = lt.view(np.int32).astype(np.int64) - cr.view(np.int32).astype(np.int64)
    assert np.all(np.abs(d) <= 1) and lt[(0x3F800000 - llo)] == 0.0
    print(f"1-ulp outputs: v_exp_f32 {e_off:.3%}, v_log_f32 {np.mean(d != 0):.3%}")


def test_trans_outside_tables():
    """Every f32 t >= 48 gives 0 <= v_exp_f32(-t) <= 2^-39 (so 256 * 2^-t is
    absorbed wherever the definition adds it), NaN propagates, log2(1) = 0."""
    import ctypes as C
    from modulations_amd import _native
    bad = C.c_longlong(-1)
    _native.check(_native.lib().tdec_selftest(0, 3, 0, 0, C.byref(bad)))
    assert bad.value == 0


def _logmap_exact(Lc, La, sf, t):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_oracle_golden import _logmap_f64_exact
    return _logmap_f64_exact(Lc, La, sf, t)


def test_logmap_gpu_siso_within_1e5_of_exact_log_map():
    """The kernel's log-MAP SISO (hardware primitives) against log-MAP with exact
    f64 Jacobian logarithms: the north star's 1e-5 (plus two f32 ulps of the
    block's largest input metric once that exceeds the f32 resolution)."""
    rng = np.random.default_rng(1)
    t, _ = O.trellis()
    for i, (sc, lsc, n) in enumerate(((1, 3, 48), (4, 3, 48), (2, 8, 212), (6, 20, 212), (3, 10, 752), (8, 40, 100))):
        Lc = (rng.standard_normal((4, 1, n)) * sc).astype(np.float32)
        La = rng.standard_normal((2, 1, n)) * lsc
        A, B = M.bcjr_max_log_map_batch(*Lc, *La, *t, n, 0.7, algo="log-map")
        RA, RB = _logmap_exact(Lc[:, 0], La[:, 0], 0.7, t)
        big = max(np.max(np.abs(Lc[0, 0] + La[0, 0])), np.max(np.abs(Lc[1, 0] + La[1, 0])))
        tol = 1e-5 if i < 3 else 1e-5 + 2 * 2.0 ** -23 * big
        assert max(np.max(np.abs(A[0] - RA)), np.max(np.abs(B[0] - RB))) <= tol, (sc, lsc, n)


# ---- the frame decoder / frame SISO in log-MAP (round 5): small batches ---------------
# One codeword per workgroup (tdec_frame.hip, ALGO 1): the pair values v(wy) + max*(U_c,
# -U_c) in the LDS table, the recursions' step with max* over the two predecessor
# (successor) classes, segments that re-run until they merge, extrinsic<1>.  Batches up
# to LM_FRAME_MAX codewords take it (decode() per frame was one lane of the throughput
# kernel: ~28 ms at N = 752); compared with the oracle's log-MAP (algo 1, the device's
# primitive tables) bit for bit, bits and L_final.
@pytest.mark.parametrize("n,rate", [(48, "1/3"), (212, "1/3"), (752, "1/2"), (848, "1/3"), (220, "2/3")])
@pytest.mark.parametrize("B,noise", [(1, 1.0), (3, 2.2), (65, 1.5)])
def test_logmap_frame_decode_matches_oracle(n, rate, B, noise):
    rng = np.random.default_rng(n * 3 + B)
    c = M.DVBRCS2_Turbo(n, rate, algo="log-map")
    info = rng.integers(0, 2, (B, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in info]).astype(np.float32)
    llr += (rng.standard_normal(llr.shape) * noise).astype(np.float32)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    t, _ = O.trellis()
    rb, rl = O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, t, algo=1, want_lfinal=True, nthreads=16)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)
    if B == 1:
        assert np.array_equal(c.decode(llr[0]), rb[0])     # decode() per frame, test.py:81


@pytest.mark.parametrize("kind", ["nan", "inf", "tiny", "huge"])
def test_logmap_frame_decode_edge_inputs(kind):
    rng = np.random.default_rng(7)
    c = M.DVBRCS2_Turbo(212, "1/3", algo="log-map")
    llr = (rng.standard_normal((3, c.n_coded)) * 2).astype(np.float32)
    if kind == "nan":
        llr[0, rng.integers(0, c.n_coded, 20)] = np.nan
        llr[2, :] = np.nan
    elif kind == "inf":
        llr[0, rng.integers(0, c.n_coded, 20)] = np.inf
        llr[1, rng.integers(0, c.n_coded, 20)] = -np.inf
    elif kind == "tiny":
        llr *= np.float32(1e-4)
    else:
        llr *= np.float32(1e4)
    bits, lf = c.decode_batch(llr, return_lfinal=True)
    t, _ = O.trellis()
    rb, rl = O.decode_batch(llr, c.N, c.punct["period"], T.puncture_matrix(c.punct), c.iterations, c.perm,
                            c.inv_perm, t, algo=1, want_lfinal=True, nthreads=8)
    assert np.array_equal(bits, rb)
    np.testing.assert_array_equal(lf, rl)


def test_logmap_frame_equals_throughput_decoder():
    """4 096 codewords through the frame decoder, 7 169 (one more than its limit,
    tdec_api.hip LM_FRAME_MAX) through the persistent throughput kernel: the same
    bits on the shared rows."""
    rng = np.random.default_rng(4097)
    c = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    base = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in rng.integers(0, 2, (32, c.k_info))])
    llr = (base[rng.integers(0, 32, 7169)] + rng.standard_normal((7169, c.n_coded)) * 1.5).astype(np.float32)
    b_frame, l_frame = c.decode_batch(llr[:4096], return_lfinal=True)
    b_tp, l_tp = c.decode_batch(llr, return_lfinal=True)
    assert np.array_equal(b_frame, b_tp[:4096])
    np.testing.assert_array_equal(l_frame, l_tp[:4096])


@pytest.mark.parametrize("n", [1, 5, 48, 212, 752, 848, 1000])
@pytest.mark.parametrize("lc", ["f32", "f64"])
def test_logmap_frame_siso_matches_oracle(n, lc):
    rng = np.random.default_rng(n + 5)
    t, _ = O.trellis()
    B = 3
    Lc = [rng.standard_normal((B, n)) * 3 for _ in range(4)]
    if lc == "f32":
        Lc = [x.astype(np.float32) for x in Lc]
    La = [rng.standard_normal((B, n)) * 9 for _ in range(2)]
    A, Bv = M.bcjr_max_log_map_batch(*Lc, *La, *t, n, 0.7, algo="log-map")
    for r in range(B):
        ra, rb = O.siso(*(x[r] for x in Lc), *(x[r] for x in La), t, 0.7, algo=1)
        np.testing.assert_array_equal(A[r], ra)
        np.testing.assert_array_equal(Bv[r], rb)
