#!/usr/bin/env python3
"""Placement study: with TDEC_VMM_ORDERS=K and TDEC_PROBE_VERBOSE=1, reserve() times
a one-iteration decode on K chunk orders of the same physical workspace chunks
(stderr), then this script times full decodes of the bench workload on the order it
kept.  python tools/vmm_orders.py [--batch 1048576 --reps 3]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd.workload import DevicePipeline, make_symbols  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = M.DVBRCS2_Turbo(752, "1/3")
    pipe = DevicePipeline(c, "16QAM", a.batch, dev)
    _, syms, n0 = make_symbols(c, a.batch, "16QAM", 2.0, 7, dev, want_info=False)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pipe.run(syms, n0)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        pipe.run(syms, n0, events=ev)
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    print(f"orders={os.environ.get('TDEC_VMM_ORDERS', '1')} decode ms per launch: " + " ".join(f"{t:.2f}" for t in ts),
          flush=True)


if __name__ == "__main__":
    main()
