"""Device-side synthetic workloads: random info bits ->
batched device encoder (encode, dvb_rcs2_turbo.py:404-462) -> labelled Gray
constellation (the reference mappers) -> complex AWGN.  Everything stays in
HBM; nothing here is timed by bench.py."""
from __future__ import annotations

import numpy as np

from . import demap as D


def noise_n0(constellation, rate, bps, ebn0_db):
    """N0 for Eb/N0 in dB with Es = mean |c|^2 (the 256QAM table is not
    unit-power: 1.0153, sdr_modem.py:195-207)."""
    es = float(np.mean(np.abs(np.asarray(constellation)) ** 2))
    return es / (rate * bps * 10 ** (ebn0_db / 10.0))


def make_symbols(codec, B, mod, ebn0_db, seed, device):
    """(info uint8 [B, 2N], received symbols complex64 [B, S], N0) on `device`.

    The coded stream of each codeword is zero-padded to whole symbols as the
    reference mappers pad (test_sdr_with_coding.py:45-86)."""
    import torch
    bps = D.MODULATIONS[mod]["bps"]
    cons = D.constellation(mod)
    rate = codec.k_info / codec.n_coded
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    info = torch.randint(0, 2, (B, codec.k_info), generator=g, device=device, dtype=torch.uint8)
    coded = codec.encode_device(info)
    n = coded.shape[1]
    S = -(-n // bps)
    if S * bps > n:
        coded = torch.nn.functional.pad(coded, (0, S * bps - n))
    w = 1 << torch.arange(bps - 1, -1, -1, device=device, dtype=torch.int32)
    labels = (coded.view(B, S, bps).to(torch.int32) * w).sum(-1)
    del coded
    table = torch.from_numpy(np.ascontiguousarray(cons.astype(np.complex64))).to(device)
    x = table[labels]
    del labels
    n0 = noise_n0(cons, rate, bps, ebn0_db)
    noise = torch.randn((B, S, 2), generator=g, device=device, dtype=torch.float32) * float(np.sqrt(n0 / 2))
    y = (x + torch.view_as_complex(noise)).contiguous()
    return info, y, n0


class DevicePipeline:
    """Fused demap -> turbo decode over device-resident symbols (the bench step).

    Buffers are sized once (tdec_reserve + planes + bits); run() is
    stream-ordered and allocation free."""

    def __init__(self, codec, mod, B, device):
        import torch
        self.codec, self.mod, self.B = codec, mod, B
        self.bps = D.MODULATIONS[mod]["bps"]
        self.cons = D.constellation(mod)
        codec.reserve(B)
        self.planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=device)
        self.bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=device)

    def run(self, syms, noise_var, stream=None, events=None):
        _, div32, nve = D.demap_mode(np.complex64, self.cons.dtype, np.float64(noise_var))
        self.codec.demap_planes_device(syms, self.cons, self.bps, nve, self.planes, div_f32=div32, stream=stream)
        if events is not None:
            events[0].record(stream)
        self.codec.decode_planes_device(self.planes, syms.shape[0], self.bits, stream=stream)
        if events is not None:
            events[1].record(stream)
        return self.bits
