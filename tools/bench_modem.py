#!/usr/bin/env python3
"""Throughput of the modem front-end kernels on one
MI355X, device-resident data, against the HBM roofline.

Every kernel here is a byte-moving pass, so each line reports algorithmic
bytes (inputs read once + outputs written once) / kernel time, timed with HIP
events on the stream the kernels run on.  One JSON line per kernel on stdout.

  python tools/bench_modem.py [--msym 32] [--reps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from modulations_amd import demap as D  # noqa: E402
from modulations_amd import modem as MM  # noqa: E402

PEAK = 8000.0   # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)


def timed(fn, reps, stream):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--msym", type=float, default=128, help="millions of symbols")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    n = int(a.msym * 1e6)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    res = []

    def report(name, ms, bytes_, unit_count, unit):
        gbs = bytes_ / ms / 1e6
        r = {"kernel": name, "ms": round(ms, 4), "GB_per_s": round(gbs, 1), "frac_hbm_peak": round(gbs / PEAK, 4),
             "bytes": bytes_, unit: round(unit_count / ms * 1e3, 1)}
        res.append(r)
        print(json.dumps(r), flush=True)

    # mapper: 256QAM, 8 label bytes in, one complex64 out per symbol
    t = D.constellation("256QAM")
    bits = torch.randint(0, 2, (8 * n,), generator=g, device=dev, dtype=torch.uint8)
    syms = torch.empty(n, dtype=torch.complex64, device=dev)
    ms = timed(lambda: MM.map_device(bits, 8, t, out=syms, stream=st), a.reps, st)
    report("k_map 256QAM", ms, 8 * n + 8 * n, n, "symbols_per_s")

    # hard demod 256QAM (axis rule): complex64 in, 8 bit bytes out
    out = torch.empty(8 * n, dtype=torch.uint8, device=dev)
    ms = timed(lambda: MM.demod_device(syms, MM.QAM_AXIS, 8, labels=MM._INV[4], scale=np.sqrt(170), out=out,
                                       stream=st), a.reps, st)
    report("k_demod 256QAM axis", ms, 8 * n + 8 * n, n, "symbols_per_s")
    assert torch.equal(out, bits)
    del bits, out

    # pulse shaping: _upsample_filter, sps 4, 101 taps -> complex128 [4n]
    taps = MM.rrc_taps(4)
    ns = n // 4
    x = syms[:ns].contiguous()
    y = torch.empty(4 * ns, dtype=torch.complex128, device=dev)
    ms = timed(lambda: MM.fir_device(x, taps, 4, 1, 50, 4 * ns, out=y, stream=st), a.reps, st)
    report("k_fir upsample x4 (101 taps)", ms, 8 * ns + 16 * 4 * ns, 4 * ns, "samples_per_s")

    # matched filter: full conv + [2d::8], Modulator (49 taps), complex128 in
    mo = MM.Modulator()
    L = len(mo.rrc_filter)
    nin = 4 * ns
    n_out = (nin + L - 1 - 2 * mo.filter_delay + 7) // 8
    z = torch.empty(n_out, dtype=torch.complex128, device=dev)
    ms = timed(lambda: MM.fir_device(y, mo.rrc_filter, 1, 8, 2 * mo.filter_delay, n_out, out=z, stream=st),
               a.reps, st)
    report("k_fir matched /8 (49 taps)", ms, 16 * nin + 16 * n_out, nin, "samples_per_s")

    # IQ: quantize complex128 -> int8 pairs (2 passes: max, convert), dequantize uint8 pairs -> complex64
    iq = torch.empty(2 * nin, dtype=torch.int8, device=dev)
    scratch = torch.empty(1, dtype=torch.int64, device=dev)
    ms = timed(lambda: MM.iq_quantize_device(y, out=iq, scratch=scratch, stream=st), a.reps, st)
    report("iq_quantize (absmax + convert)", ms, 2 * 16 * nin + 2 * nin, nin, "samples_per_s")
    back = torch.empty(nin, dtype=torch.complex64, device=dev)
    ms = timed(lambda: MM.iq_dequantize_device(iq.view(torch.uint8), out=back, stream=st), a.reps, st)
    report("k_dequantize", ms, 2 * nin + 8 * nin, nin, "samples_per_s")


if __name__ == "__main__":
    main()
