#!/usr/bin/env python3
"""A/B of the two SISO mappings on the same inputs:
per-lane (k_siso_batch: one codeword per lane, 64 per wave) against the north
star's state-per-lane prototype (k_siso_spl: one state per lane, 4 codewords
per wave, cross-lane exchanges every step), bcjr_max_log_map over B codewords
of N=752 couples.  Kernel times come from `rocprofv3 --kernel-trace --stats`
around this script (the host API also copies the rows over PCIe); the script
checks the two outputs are identical and prints wall times.

  rocprofv3 --kernel-trace --stats -d out -o ab -- python tools/ab_siso.py [--batch 131072]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd import tables as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=131072)
    ap.add_argument("--n", type=int, default=752)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    B, n = a.batch, a.n
    Lc = (rng.standard_normal((4, B, n)) * 3).astype(np.float32)
    La = rng.standard_normal((2, B, n)) * 6
    tabs = T.trellis_tables()[:5]
    out = {}
    for mode in ("0", "1", "0", "1")[: 2 * a.reps]:
        os.environ["TDEC_SISO_SPL"] = mode
        t0 = time.perf_counter()
        r = M.bcjr_max_log_map_batch(*Lc, *La, *tabs, n, 0.7)
        dt = time.perf_counter() - t0
        print(f"{'state-per-lane' if mode == '1' else 'per-lane      '} wall {dt:.3f} s (PCIe-inclusive)", flush=True)
        out[mode] = r
    same = all(np.array_equal(x, y) for x, y in zip(out["0"], out["1"]))
    print("identical outputs:", same)
    assert same


if __name__ == "__main__":
    main()
