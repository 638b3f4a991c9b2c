"""Fused demap + decode (tdec_demap_decode_dev, k_turbo_decode_syms): every
decoder wave demaps its own tile into a per-wave plane buffer.  Its bits and
L_final must be those of the two-launch path (k_demap_planes -> planes ->
k_turbo_decode), which the other tests pin to the oracle, for every
instantiated configuration, ragged batches and batches past the resident waves
(the persistent loop reuses each wave's plane buffer, so stale L1 lines would
show up here), plus an oracle spot check."""
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


def _two_launch(codec, mod, syms, n0, lfinal=False):
    B = syms.shape[0]
    pipe = DevicePipeline(codec, mod, B, "cuda", fused=False)
    cons = D.constellation(mod)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device="cuda")
    lf = torch.empty((B, codec.k_info), dtype=torch.float64, device="cuda") if lfinal else None
    codec.demap_planes_device(syms, cons, pipe.bps, nve, pipe.planes, div_f32=div32)
    codec.decode_planes_device(pipe.planes, B, bits, lfinal=lf)
    return bits, lf


@pytest.mark.parametrize("mod,n,rate,algo,B", [("16QAM", 752, "1/3", "max-log", 4099),
                                              ("256QAM", 752, "1/3", "max-log", 1000),
                                              ("QPSK", 212, "1/3", "max-log", 777),
                                              ("8PSK", 752, "1/2", "log-map", 300),
                                              ("16QAM", 48, "1/2", "max-log", 65),
                                              ("16QAM", 212, "2/3", "max-log", 130)])
def test_fused_equals_two_launch_path(mod, n, rate, algo, B):
    codec = M.DVBRCS2_Turbo(n, rate, algo=algo)
    cons = D.constellation(mod)
    bps = D.MODULATIONS[mod]["bps"]
    assert codec.fused_available(cons, bps)
    _, syms, n0 = make_symbols(codec, B, mod, 2.0, 123, "cuda", want_info=False)
    ref_bits, ref_lf = _two_launch(codec, mod, syms, n0, lfinal=True)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    codec.reserve_fused(B)
    bits = torch.empty_like(ref_bits)
    lf = torch.empty_like(ref_lf)
    codec.demap_decode_device(syms, cons, bps, nve, bits, lfinal=lf, div_f32=div32)
    torch.cuda.synchronize()
    assert torch.equal(bits, ref_bits)
    assert torch.equal(lf, ref_lf)


def test_fused_full_size_wraps_and_matches_oracle():
    codec = M.DVBRCS2_Turbo(752, "1/3")
    B = 140_000                              # > 2048 resident waves x 64: each wave reuses its plane buffer
    _, syms, n0 = make_symbols(codec, B, "16QAM", 2.0, 77, "cuda", want_info=False)
    fused = DevicePipeline(codec, "16QAM", B, "cuda", fused=True)
    assert fused.fused
    b1 = fused.run(syms, n0).clone()
    ref, _ = _two_launch(codec, "16QAM", syms, n0)
    torch.cuda.synchronize()
    assert torch.equal(b1, ref)
    cons = D.constellation("16QAM")
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    idx = [0, 63, 64, 131_071, 131_072, B - 1]
    rows = syms[idx].cpu().numpy()
    llr = np.stack([-O.demap(r, cons, 4, nve, div_f32=div32)[:codec.n_coded] for r in rows]).astype(np.float32)
    t, _ = O.trellis()
    rb = O.decode_batch(llr, 752, 1, T.puncture_matrix(codec.punct), 8, codec.perm, codec.inv_perm, t)
    assert np.array_equal(b1[idx].cpu().numpy(), rb)


def test_fused_unavailable_configurations_fall_back():
    codec = M.DVBRCS2_Turbo(212, "1/3")
    assert not codec.fused_available(D.constellation("64QAM"), 6)
    B = 200
    _, syms, n0 = make_symbols(codec, B, "64QAM", 3.0, 5, "cuda", want_info=False)
    pipe = DevicePipeline(codec, "64QAM", B, "cuda", fused=True)
    assert not pipe.fused
    ref, _ = _two_launch(codec, "64QAM", syms, n0)
    assert torch.equal(pipe.run(syms, n0), ref)
