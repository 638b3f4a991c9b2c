"""Device-side synthetic workloads: counter-based (Philox)
info bits -> batched device encoder (encode, dvb_rcs2_turbo.py:404-462) ->
labelled Gray constellation (the reference mappers) -> complex AWGN, and the
per-codeword error counters of a BER point.  Everything stays in HBM; nothing
here is timed by bench.py."""
from __future__ import annotations

import numpy as np

from . import demap as D


def noise_n0(constellation, rate, bps, ebn0_db):
    """N0 for Eb/N0 in dB with Es = mean |c|^2 (the 256QAM table is not
    unit-power: 1.0153, sdr_modem.py:195-207)."""
    es = float(np.mean(np.abs(np.asarray(constellation)) ** 2))
    return es / (rate * bps * 10 ** (ebn0_db / 10.0))


def make_symbols(codec, B, mod, ebn0_db, seed, device, cw0=0, want_info=True):
    """(info uint8 [B, 2N] or None, received symbols complex64 [B, S], N0) on `device`.

    One launch of the counter-based generator (tdec_workload_dev): Philox info
    bits of GLOBAL codewords cw0 .. cw0+B-1 -> the LDS-staged encoder ->
    labelled Gray constellation (bps coded bits per label, MSB first, the last
    symbol zero-padded as the reference mappers pad, test_sdr_with_coding.py:45-86)
    -> complex AWGN with per-dimension variance N0/2.  Codeword g's data is the
    same whichever batch or rank generates it."""
    import torch
    from . import _native as _n
    bps = D.MODULATIONS[mod]["bps"]
    cons = D.constellation(mod)
    rate = codec.k_info / codec.n_coded
    h = codec.handle
    S = -(-h.enc_len // bps)
    n0 = noise_n0(cons, rate, bps, ebn0_db)
    table = np.ascontiguousarray(cons.astype(np.complex64)).view(np.float32)
    syms = torch.empty((B, S), dtype=torch.complex64, device=device)
    info = torch.empty((B, codec.k_info), dtype=torch.uint8, device=device) if want_info else None
    h.call("tdec_workload_dev", int(B), int(cw0), int(seed) & 0xFFFFFFFFFFFFFFFF, _n.ptr(table), len(cons), bps,
           float(np.sqrt(n0 / 2)), _n.ptr(syms), _n.ptr(info), codec._stream(None))
    return info, syms, n0


def info_bits(codec, B, seed, device, cw0=0):
    """The info bits make_symbols encodes, uint8 [B, 2N]."""
    import torch
    info = torch.empty((B, codec.k_info), dtype=torch.uint8, device=device)
    codec.handle.call("tdec_info_bits_dev", int(B), int(cw0), int(seed) & 0xFFFFFFFFFFFFFFFF,
                      _ptr(info), codec._stream(None))
    return info


def count_errors(codec, bits, seed, cw0=0):
    """Bit errors per codeword (int32 [B]) of decoded rows against the
    counter-based info bits of global codewords cw0 .. cw0+B-1."""
    import torch
    B = bits.shape[0]
    if bits.dtype != torch.int32 or not bits.is_contiguous() or tuple(bits.shape) != (B, codec.k_info):
        raise ValueError("bits must be a contiguous int32 [B, 2N] tensor")
    errs = torch.empty(B, dtype=torch.int32, device=bits.device)
    codec.handle.call("tdec_count_errors_dev", int(B), int(cw0), int(seed) & 0xFFFFFFFFFFFFFFFF, _ptr(bits),
                      _ptr(errs), codec._stream(None))
    return errs


def _ptr(t):
    from . import _native as _n
    return _n.ptr(t)


class DevicePipeline:
    """Demap -> turbo decode over device-resident symbols (the bench step).

    Default: the two launches k_demap_planes + k_turbo_decode over a plane
    buffer.  fused=True uses the one-launch k_turbo_decode_syms (each decoder
    wave demaps its next tile between the SISOs of the current one) where the
    handle has it; the bits are the same either way.  The fused launch measured
    3-4 % SLOWER on MI355X (294 vs 285 ms per 1 M codewords): a
    wave that demaps is not streaming, and at two waves per SIMD the decoder
    needs every wave streaming to keep HBM busy.  Buffers are sized once; run()
    is stream-ordered and allocation free."""

    def __init__(self, codec, mod, B, device, fused=False, overlap=False, gate=True):
        import torch
        self.codec, self.mod, self.B = codec, mod, B
        self.bps = D.MODULATIONS[mod]["bps"]
        self.cons = D.constellation(mod)
        self.fused = bool(fused) and codec.fused_available(self.cons, self.bps)
        self.overlap = bool(overlap) and not self.fused
        if self.fused:
            codec.reserve_fused(B)
            self.planes = None
        else:
            codec.reserve(B)
            self.planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=device)
        self.bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=device)
        if self.overlap:
            # Batch i+1's demap runs on its own handle (handles order only their own
            # buffers), its own low-priority stream and the other plane buffer, so
            # it can start as soon as batch i's persistent decoder waves begin to
            # retire (tail of the persistent launch) instead of after
            # the last one.  The decode runs on a high-priority stream, so a decode
            # and a demap that become ready together dispatch the decode first.
            import copy
            self.demapper = copy.copy(codec)
            self.demapper._h = None
            self.planes_db = [self.planes, torch.empty_like(self.planes)]
            self.s_demap = torch.cuda.Stream(device=device, priority=0)
            self.s_decode = torch.cuda.Stream(device=device, priority=-1)
            self.demap_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.decode_done = [torch.cuda.Event(), torch.cuda.Event()]
            self.step = 0
            self.gate = bool(gate)

    def run(self, syms, noise_var, stream=None, events=None, syms_ready=None):
        """One batch: demap -> decode, stream-ordered on `stream` (its bits are ready
        for work queued on `stream` afterwards).  With overlap=True, `syms_ready`
        (an event after which `syms` is valid) lets the demap start before the
        previous batch's decode has finished; without it the demap waits for
        everything queued on `stream`, i.e. no overlap."""
        _, div32, nve = D.demap_mode(np.complex64, self.cons.dtype, np.float64(noise_var))
        bits = self.bits[:syms.shape[0]]          # the first rows: a contiguous view
        if self.overlap:
            import torch
            stream = torch.cuda.current_stream() if stream is None else stream
            b = self.step & 1
            sd, sk = self.s_demap, self.s_decode
            if self.step >= 2:
                sd.wait_event(self.decode_done[b])      # planes[b]'s last reader (batch i-2)
            if syms_ready is not None:
                sd.wait_event(syms_ready)
            else:
                sd.wait_stream(stream)
            if self.gate:
                self.codec.tail_gate(sd)                # batch i-1's decode is in its tail
            self.demapper.demap_planes_device(syms, self.cons, self.bps, nve, self.planes_db[b], div_f32=div32,
                                              stream=sd)
            self.demap_done[b].record(sd)
            sk.wait_stream(stream)                      # earlier readers of bits on the caller's stream
            sk.wait_event(self.demap_done[b])
            if events is not None:
                events[0].record(sk)
            self.codec.decode_planes_device(self.planes_db[b], syms.shape[0], bits, stream=sk)
            if events is not None:
                events[1].record(sk)
            self.decode_done[b].record(sk)
            stream.wait_event(self.decode_done[b])
            self.step += 1
            return bits
        if self.fused:
            if events is not None:
                events[0].record(stream)
            self.codec.demap_decode_device(syms, self.cons, self.bps, nve, bits, div_f32=div32, stream=stream)
        else:
            self.codec.demap_planes_device(syms, self.cons, self.bps, nve, self.planes, div_f32=div32,
                                           stream=stream)
            if events is not None:
                events[0].record(stream)
            self.codec.decode_planes_device(self.planes, syms.shape[0], bits, stream=stream)
        if events is not None:
            events[1].record(stream)
        return bits
