"""Counter-based device workload generation (tdec_workload_dev,
tdec_info_bits_dev, tdec_count_errors_dev) and the
multi-rank paths that rely on it (bench.py --gpus N, the BER sweep).

* info bits == the host Philox4x32-10 restatement (oracle/workload_ref.py), bit for bit;
* noise-free symbols == the oracle's encode (dvb_rcs2_turbo.py:404-462) mapped
  through the reference constellation, zero-padded to whole symbols;
* noise == the host Box-Muller of the same counters within f32 rounding;
* any split of the global codeword range into batches gives the same symbols;
* error counters == (decoded != info) row sums;
* bench.py --gpus 2 spawns two ranks itself (gloo, both on GPU 0) and reports
  n_gpus 2 with the counters of a one-rank run over the same codewords;
* a 2-rank BER point equals the 1-rank point.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from oracle import workload_ref as W  # noqa: E402
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402
from modulations_amd.workload import count_errors, info_bits, make_symbols  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("n", [48, 212, 752, 848])
def test_info_bits_match_host_philox(n):
    c = M.DVBRCS2_Turbo(n, "1/3")
    seed, cw0, B = 0xDEADBEEF12345, 98_765, 300
    got = info_bits(c, B, seed, "cuda", cw0=cw0)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), W.info_bits(np.arange(cw0, cw0 + B), n, seed))


@pytest.mark.parametrize("mod,n,rate", [("16QAM", 752, "1/3"), ("8PSK", 752, "1/2"), ("QPSK", 212, "1/3"),
                                        ("256QAM", 752, "1/3"), ("BPSK", 48, "2/3"), ("64QAM", 64, "3/4")])
def test_noise_free_symbols_are_the_encoded_constellation(mod, n, rate):
    c = M.DVBRCS2_Turbo(n, rate)
    bps = D.MODULATIONS[mod]["bps"]
    cons = D.constellation(mod).astype(np.complex64)
    B, seed = 130, 77
    info, syms, _ = make_symbols(c, B, mod, 1000.0, seed, "cuda", cw0=5)      # sigma ~ 0: labels exact below
    info = info.cpu().numpy()
    assert np.array_equal(info, W.info_bits(np.arange(5, 5 + B), n, seed))
    t, G = O.trellis()
    pm = T.puncture_matrix(c.punct)
    coded = np.stack([O.encode(b, n, c.punct["period"], pm, c.perm, t, G) for b in info])
    S = -(-coded.shape[1] // bps)
    padded = np.pad(coded, ((0, 0), (0, S * bps - coded.shape[1])))
    labels = (padded.reshape(B, S, bps) * (1 << np.arange(bps - 1, -1, -1))).sum(-1)
    want = cons[labels]
    got = syms.cpu().numpy()
    assert got.shape == (B, S)
    # the noise at 1000 dB is ~1e-50 of the signal: every point rounds to the table value
    assert np.array_equal(got, want)


def test_noise_matches_host_box_muller_and_split_invariance():
    c = M.DVBRCS2_Turbo(752, "1/3")
    seed, B = 4242, 1000
    _, full, n0 = make_symbols(c, B, "16QAM", 2.0, seed, "cuda", cw0=0, want_info=False)
    a = make_symbols(c, 400, "16QAM", 2.0, seed, "cuda", cw0=0, want_info=False)[1]
    b = make_symbols(c, 600, "16QAM", 2.0, seed, "cuda", cw0=400, want_info=False)[1]
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([a, b]), full)
    info, clean, _ = make_symbols(c, 64, "16QAM", 1000.0, seed, "cuda", cw0=0)
    noise = full[:64].cpu().numpy().astype(np.complex128) - clean.cpu().numpy()
    ref = W.awgn(np.arange(64), full.shape[1], seed, np.sqrt(n0 / 2))
    assert np.max(np.abs(noise - ref)) < 2e-5


def test_staged_encoder_matches_row_kernel_for_all_block_sizes():
    rng = np.random.default_rng(9)
    t, G = O.trellis()
    for n in (48, 64, 212, 220, 424, 752, 848):
        for rate in ("1/3", "1/2", "2/3", "3/4"):
            c = M.DVBRCS2_Turbo(n, rate)
            bits = rng.integers(0, 2, (70, c.k_info)).astype(np.uint8)
            got = c.encode_device(torch.from_numpy(bits).cuda()).cpu().numpy()
            pm = T.puncture_matrix(c.punct)
            want = np.stack([O.encode(b, n, c.punct["period"], pm, c.perm, t, G) for b in bits[:9]])
            assert np.array_equal(got[:9], want), (n, rate)
            assert np.array_equal(got[-1], O.encode(bits[-1], n, c.punct["period"], pm, c.perm, t, G))


def test_count_errors():
    c = M.DVBRCS2_Turbo(212, "1/3")
    B, seed, cw0 = 500, 99, 1234
    info = info_bits(c, B, seed, "cuda", cw0=cw0).to(torch.int32)
    flip = (torch.rand((B, c.k_info), device="cuda") < 0.01).to(torch.int32)
    flip[::7] = 0
    dec = (info ^ flip).contiguous()
    e = count_errors(c, dec, seed, cw0=cw0)
    torch.cuda.synchronize()
    assert torch.equal(e.cpu(), flip.sum(1).to(torch.int32).cpu())


def _run(cmd, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_bench_spawns_ranks_and_matches_single_rank_counters():
    common = ["--steps", "1", "--warmup", "1", "--no-cpu", "--n", "212", "--mod", "QPSK", "--ebn0", "1.0"]
    two = json.loads(_run([sys.executable, "bench.py", "--gpus", "2", "--all-on-device0", "--dist-backend", "gloo",
                           "--batch", "4096", *common]).strip().splitlines()[-1])
    one = json.loads(_run([sys.executable, "bench.py", "--gpus", "1", "--batch", "8192", *common])
                     .strip().splitlines()[-1])
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["ber"] == one["ber"]
    assert two["ber"]["codewords"] == 8192


def test_bench_rccl_path_single_rank_under_torchrun():
    """The driver's multi-GPU launch (torchrun, one rank per GPU, backend nccl = RCCL,
    init_process_group(device_id=...), barrier, all-reduce of the counters and of the
    max time) on the one GPU a test box has: one rank with --dist-always.  Counters
    equal the plain single-process run's."""
    # (no "--n": torchrun's own parser takes it for an abbreviation of its options)
    common = ["--steps", "1", "--warmup", "1", "--no-cpu", "--mod", "QPSK", "--ebn0", "1.0", "--batch", "8192"]
    port = str(28500 + os.getpid() % 1000)
    rccl = json.loads(_run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                            "--master-addr", "127.0.0.1", "--master-port", port, "bench.py", "--gpus", "1",
                            "--dist-always", *common]).strip().splitlines()[-1])
    one = json.loads(_run([sys.executable, "bench.py", "--gpus", "1", *common]).strip().splitlines()[-1])
    assert rccl["n_gpus"] == 1 and rccl["value"] > 0
    assert rccl["ber"] == one["ber"] and rccl["ber"]["codewords"] == 8192


def test_ber_point_independent_of_world_size(tmp_path):
    args = ["-m", "modulations_amd.ber", "--mod", "QPSK", "--couples", "212", "--rate", "1/3", "--ebn0", "0.5",
            "--codewords", "5000", "--batch", "1500", "--seed", "7"]
    one = json.loads(_run([sys.executable, *args]).strip().splitlines()[-1])
    port = str(29500 + os.getpid() % 1000)
    two = json.loads(_run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                           "--master-addr", "127.0.0.1", "--master-port", port, *args,
                           "--dist-backend", "gloo", "--all-on-device0"]).strip().splitlines()[-1])
    for k in ("codewords", "bit_errors", "frame_errors"):
        assert one[k] == two[k], k
    assert one["codewords"] == 5000 and one["bit_errors"] > 0


def test_overlapped_pipeline_gives_the_serial_bits():
    """DevicePipeline(overlap=True) (next batch's demap on its own handle, stream and
    plane buffer) decodes every batch to the serial pipeline's bits, batch after
    batch with alternating plane buffers and different symbols per batch."""
    from modulations_amd.workload import DevicePipeline
    c = M.DVBRCS2_Turbo(212, "1/3")
    B = 4096
    serial = DevicePipeline(c, "16QAM", B, torch.device("cuda", 0))
    c2 = M.DVBRCS2_Turbo(212, "1/3")
    ovl = DevicePipeline(c2, "16QAM", B, torch.device("cuda", 0), overlap=True)
    batches = [make_symbols(c, B, "16QAM", 2.0, 1234, "cuda", cw0=j * B, want_info=False) for j in range(3)]
    ready = torch.cuda.Event()
    ready.record()
    want, got = [], []
    for _, syms, n0 in batches:
        want.append(serial.run(syms, n0).clone())
    for _, syms, n0 in batches:
        got.append(ovl.run(syms, n0, syms_ready=ready).clone())   # clone on the caller's stream: after the decode
    torch.cuda.synchronize()
    for w, g in zip(want, got):
        assert torch.equal(w, g)
