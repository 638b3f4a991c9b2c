#!/usr/bin/env python3
"""Workspace-placement study: one process,
TDEC_PLACEMENT_PROBE=0, K decoder handles each with its own freshly allocated
full-GPU workspace (all kept alive, so every one lands somewhere else in HBM),
the same device-resident planes, one timed decode per handle per round.  Run
bare for the timings, and under separate `rocprofv3 --pmc` passes for the
address-translation and memory-latency counters of each dispatch:

  python tools/placement_counters.py [--handles 8] [--rounds 2] [--batch 262144]
"""
import argparse
import os
import sys

os.environ["TDEC_PLACEMENT_PROBE"] = "0"
import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from modulations_amd import demap as D  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd.workload import make_symbols  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--handles", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--batch", type=int, default=262144)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.batch
    codec = M.DVBRCS2_Turbo(752, "1/3")
    _, syms, n0 = make_symbols(codec, B, "16QAM", 2.0, 99, dev, want_info=False)
    cons = D.constellation("16QAM")
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    codec.reserve(B)
    planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=dev)
    codec.demap_planes_device(syms, cons, 4, nve, planes, div_f32=div32)
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=dev)
    handles = []
    for i in range(a.handles):
        c = M.DVBRCS2_Turbo(752, "1/3")
        c.reserve(B)
        handles.append(c)
    st = torch.cuda.current_stream()
    ref = None
    times = np.zeros((a.rounds, a.handles))
    for r in range(a.rounds):
        for i, c in enumerate(handles):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            c.decode_planes_device(planes, B, bits)
            e1.record(st)
            torch.cuda.synchronize()
            times[r, i] = e0.elapsed_time(e1)
            if ref is None:
                ref = bits.clone()
            assert torch.equal(bits, ref)
    for i in range(a.handles):
        print(f"handle {i}: " + " ".join(f"{t:7.2f}" for t in times[:, i]) + " ms", flush=True)


if __name__ == "__main__":
    main()
