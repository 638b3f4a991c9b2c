"""Size-independent properties at the bench's full size (N=752 couples,
rate 1/3, 8 iterations, batches past the resident-wave count so the
persistent tile loop wraps), where the oracle cannot check every codeword:

* determinism, batch-order invariance and shard equivalence (one launch ==
  the concatenation of launches over its shards) -- bit for bit;
* the timed kernel itself (k_turbo_decode: batches above the small-batch
  decoders' limit) against the oracle on 4 096 rows of each full-size batch --
  the first 2 048 (32 tiles) and 2 048 spread over the whole batch, so rows of
  every round of the persistent tile loop are checked -- bits AND L_final;
* the fused demap+decode pipeline == compute_llr -> float32 -> decode;
* with a true permutation (valid-perm mode) a noise-free batch decodes to its
  info bits exactly (encode -> decode round trip).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402
from modulations_amd.workload import DevicePipeline, make_symbols  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _oracle_bits(codec, llr_rows, want_lfinal=False):
    t, _ = O.trellis()
    return O.decode_batch(llr_rows, codec.N, codec.punct["period"], T.puncture_matrix(codec.punct),
                          codec.iterations, codec.perm, codec.inv_perm, t, nthreads=16, want_lfinal=want_lfinal)


def _host_llr_rows(codec, syms_rows, mod, n0):
    """compute_llr (the C oracle's restatement) -> decoder sign -> float32, per row."""
    cons = D.constellation(mod)
    bps = D.MODULATIONS[mod]["bps"]
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    R, S = syms_rows.shape
    llr = -O.demap(np.ascontiguousarray(syms_rows).reshape(-1), cons, bps, nve, div_f32=div32)
    return np.ascontiguousarray(llr.reshape(R, S * bps)[:, :codec.n_coded]).astype(np.float32)


def _check_throughput_kernel_vs_oracle(codec, pipe, syms, B, n0, mod):
    """Re-decode the pipeline's planes (B > the small-batch limit, so
    k_turbo_decode runs) with L_final and compare 4 096 rows with the oracle."""
    lf = torch.empty((B, codec.k_info), dtype=torch.float64, device=syms.device)
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=syms.device)
    codec.decode_planes_device(pipe.planes, B, bits, lfinal=lf)
    torch.cuda.synchronize()
    idx = np.unique(np.concatenate([np.arange(2048), np.linspace(2048, B - 1, 2048).astype(np.int64)]))
    assert len(idx) >= 4096 and idx[-1] == B - 1
    ti = torch.as_tensor(idx, device=syms.device)
    llr = _host_llr_rows(codec, syms[ti].cpu().numpy(), mod, n0)
    rb, rl = _oracle_bits(codec, llr, want_lfinal=True)
    assert np.array_equal(bits[ti].cpu().numpy(), rb)
    np.testing.assert_array_equal(lf[ti].cpu().numpy(), rl)
    return bits


def test_full_size_pipeline_properties():
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(752, "1/3")
    B = 150_000                               # > resident waves x 64 -> the tile loop wraps
    info, syms, n0 = make_symbols(codec, B, "16QAM", 2.0, 7, dev)
    pipe = DevicePipeline(codec, "16QAM", B, dev)
    b1 = pipe.run(syms, n0).clone()
    b2 = pipe.run(syms, n0).clone()
    torch.cuda.synchronize()
    assert torch.equal(b1, b2)                                     # deterministic
    # shards: two launches over halves give the same bits
    h = B // 2 + 13
    p2 = DevicePipeline(codec, "16QAM", B - h, dev)
    pa = DevicePipeline(codec, "16QAM", h, dev)
    ba = pa.run(syms[:h].contiguous(), n0).clone()
    bb = p2.run(syms[h:].contiguous(), n0).clone()
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([ba, bb]), b1)
    # the timed kernel against the oracle: 4 096 rows, bits and L_final
    bt = _check_throughput_kernel_vs_oracle(codec, pipe, syms, B, n0, "16QAM")
    assert torch.equal(bt, b1)
    # batch-order invariance of the throughput kernel (16 384 > the small-batch limit)
    perm = torch.randperm(16384, device=dev)
    pp = DevicePipeline(codec, "16QAM", 16384, dev)
    bp = pp.run(syms[:16384][perm].contiguous(), n0)
    torch.cuda.synchronize()
    assert torch.equal(bp, b1[:16384][perm])
    # cross-decoder: the frame decoder (a 2 048-row call) gives the throughput
    # kernel's bits; the fused pipeline == compute_llr_device -> f32 -> decode_device
    llr_dev = D.compute_llr_device(syms[:2048].contiguous(), "16QAM", np.float64(n0), sign=-1)
    llr32 = llr_dev.view(2048, -1)[:, :codec.n_coded].to(torch.float32).contiguous()
    bd = codec.decode_device(llr32)
    torch.cuda.synchronize()
    assert torch.equal(bd, b1[:2048])


def test_valid_perm_round_trip_full_size():
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(752, "1/3", interleaver="valid-perm")
    B = 20_000
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    info = torch.randint(0, 2, (B, codec.k_info), generator=g, device=dev, dtype=torch.uint8)
    coded = codec.encode_device(info)
    llr = (1.0 - 2.0 * coded.to(torch.float32)) * 8.0
    bits = codec.decode_device(llr.contiguous())
    torch.cuda.synchronize()
    assert torch.equal(bits.to(torch.uint8), info)


def test_reference_interleaver_error_floor_is_deterministic():
    """Noise-free decoding with the reference interleaver leaves errors (SURVEY
    fact 3); over many codewords the count is reproducible and matches the oracle
    on a sample."""
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(212, "1/3")
    B = 9000
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    info = torch.randint(0, 2, (B, codec.k_info), generator=g, device=dev, dtype=torch.uint8)
    llr = ((1.0 - 2.0 * codec.encode_device(info).to(torch.float32)) * 20.0).contiguous()
    bits = codec.decode_device(llr)
    torch.cuda.synchronize()
    errs = (bits.to(torch.uint8) != info).sum(1).cpu().numpy()
    assert errs.min() > 0
    sample = [0, 4500, 8999]
    assert np.array_equal(bits[sample].cpu().numpy(), _oracle_bits(codec, llr[sample].cpu().numpy()))


@pytest.mark.parametrize("n,mod", [(212, "QPSK"), (220, "16QAM")])
def test_ragged_checkpoint_windows_full_size(n, mod):
    """N not a multiple of the max-log decoder's 8-step checkpoint interval
    (ragged top window in siso8), a batch past the resident-wave count (the
    persistent tile loop wraps) and not a multiple of 64: deterministic, and the
    first / middle / last codewords equal the oracle's."""
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(n, "1/3")
    assert codec.N % 8 != 0
    B = 140_001
    _, syms, n0 = make_symbols(codec, B, mod, 1.5, 21, dev, want_info=False)
    pipe = DevicePipeline(codec, mod, B, dev)
    b1 = pipe.run(syms, n0).clone()
    b2 = pipe.run(syms, n0).clone()
    torch.cuda.synchronize()
    assert torch.equal(b1, b2)
    # the timed kernel against the oracle: 4 096 rows (incl. the last, ragged tile), bits and L_final
    assert torch.equal(_check_throughput_kernel_vs_oracle(codec, pipe, syms, B, n0, mod), b1)


@pytest.mark.parametrize("n,mod,B", [(212, "QPSK", 102_400), (220, "16QAM", 100_003), (752, "16QAM", 70_001)])
def test_one_round_batches_vs_oracle(n, mod, B):
    """Batches of more 64-codeword tiles than SIMDs but fewer than resident waves
    (one round of the tile loop, some SIMDs with two waves and some with one):
    configs[1]'s shape, a ragged N with a partial last tile, and N = 752 -- 4 096
    rows against the oracle, bits and L_final.  (These batch shapes were the test
    of round 6's sub-tile units, which lost and were removed.)"""
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(n, "1/3")
    _, syms, n0 = make_symbols(codec, B, mod, 1.5, 23, dev, want_info=False)
    pipe = DevicePipeline(codec, mod, B, dev)
    b1 = pipe.run(syms, n0).clone()
    torch.cuda.synchronize()
    assert torch.equal(_check_throughput_kernel_vs_oracle(codec, pipe, syms, B, n0, mod), b1)
