#!/usr/bin/env python3
"""Placement sensitivity probe of k_turbo_decode.

Each trial shifts where the next allocations land (a dummy allocation of a
random size), then allocates fresh planes (a copy of the same inputs) and/or a
fresh decoder workspace, times one decode and frees everything.  Which buffer
moves is selected by --move: planes, ws or both.

  python tools/placement.py [--batch 262144] [--trials 8] [--move both]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd.workload import make_symbols  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--trials", type=int, default=8)
    ap.add_argument("--move", default="both", choices=["planes", "ws", "both"])
    ap.add_argument("--shifts", default="", help="le_kb:ck_kb,... workspace-internal offsets to cycle through")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    B = a.batch
    codec = M.DVBRCS2_Turbo(752, "1/3")
    info, syms, n0 = make_symbols(codec, B, "16QAM", 2.0, 99, dev)
    cons = D.constellation("16QAM")
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=dev)
    codec.reserve(B)
    codec.demap_planes_device(syms, cons, 4, nve, planes, div_f32=div32)
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    ref = None
    shifts = [tuple(x.split(":")) for x in a.shifts.split(",")] if a.shifts else [("0", "0")]
    for t in range(a.trials * len(shifts)):
        le_kb, ck_kb = shifts[t % len(shifts)]
        os.environ["TDEC_LE_SHIFT_KB"], os.environ["TDEC_CK_SHIFT_KB"] = le_kb, ck_kb
        gb = float(rng.uniform(0, 6))
        dummy = torch.empty(int(gb * 2**30), dtype=torch.uint8, device=dev)
        p = planes.clone() if a.move in ("planes", "both") else planes
        c = M.DVBRCS2_Turbo(752, "1/3") if a.move in ("ws", "both") else codec
        c.reserve(B)
        ms = []
        for rep in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            c.decode_planes_device(p, B, bits)
            e1.record(st)
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        same = ref is None or torch.equal(bits, ref)
        ref = bits.clone() if ref is None else ref
        print(f"trial {t}: shift le {le_kb} KiB ck {ck_kb} KiB  dummy {gb:4.2f} GiB  decode {ms[1]:7.2f} ms  same={same}",
              flush=True)
        del dummy, p, c
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
