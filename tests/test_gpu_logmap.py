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


def _oracle(codec, llr, algo=1):
    t, _ = O.trellis()
    return O.decode_batch(llr, codec.N, codec.punct["period"], T.puncture_matrix(codec.punct), codec.iterations,
                          codec.perm, codec.inv_perm, t, algo=algo, nthreads=8)


def _host_llrs(codec, syms_rows, mod, n0):
    cons = D.constellation(mod)
    bps = D.MODULATIONS[mod]["bps"]
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    return np.stack([-O.demap(r, cons, bps, nve, div_f32=div32)[:codec.n_coded] for r in syms_rows]).astype(np.float32)


def test_8psk_demap_planes_to_logmap_decode_n752_r12():
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(752, "1/2", algo="log-map")
    assert codec.n_coded == 3008
    B = 96
    info, syms, n0 = make_symbols(codec, B, "8PSK", 3.0, 11, dev)
    assert syms.shape == (B, 1003)                        # 3008 bits + 1 zero pad bit -> 1003 symbols
    pipe = DevicePipeline(codec, "8PSK", B, dev)
    bits = pipe.run(syms, n0).clone()
    torch.cuda.synchronize()
    llr = _host_llrs(codec, syms.cpu().numpy(), "8PSK", n0)
    assert np.array_equal(bits.cpu().numpy(), _oracle(codec, llr))
    # and through the LLR-row boundary (host demap -> f32 -> decode): the same bits
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
