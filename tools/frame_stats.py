#!/usr/bin/env python3
"""Segment statistics of the frame decoder (tdec_frame.hip) on real decoder
inputs: blocks of 4 recursion steps per SISO and direction in phase A, in the
fix-up rounds and in the second pass, and rounds per SISO.  Needs the
measurement build:  python -m modulations_amd.build --variant frstats TDEC_FR_STATS=1
then  python tools/frame_stats.py [N rate ebn0 B]   (16QAM symbols, device generator)."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["TDEC_LIB_VARIANT"] = os.environ.get("FRSTATS_VARIANT", "frstats")   # frtime: TDEC_FR_STATS=2
import torch  # noqa: E402,F401  (the HIP runtime torch loads: see tools/hip_probe.py)
from modulations_amd import _native as _n  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 752
    rate = sys.argv[2] if len(sys.argv) > 2 else "1/3"
    ebn0 = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    lib = _n.lib()
    c = M.DVBRCS2_Turbo(n, rate)
    rng = np.random.default_rng(1)
    info = rng.integers(0, 2, (B, c.k_info))
    Rn = {"1/3": 1 / 3, "1/2": 1 / 2, "2/3": 2 / 3, "3/4": 3 / 4}[rate]
    n0 = 1.0 / (Rn * 2 * 10 ** (ebn0 / 10))
    coded = np.stack([c.encode(b) for b in info])
    llr = ((1 - 2.0 * coded) * 2 / n0 * np.sqrt(2) / np.sqrt(2)
           + rng.standard_normal(coded.shape) * np.sqrt(2 / n0)).astype(np.float32)   # BPSK-equivalent LLRs
    out = (C.c_ulonglong * 8)()
    c.decode_batch(llr)            # creates the handle (HIP initialised), warms up
    lib.tdec_frame_stats(out)      # reset
    c.decode_batch(llr)
    lib.tdec_frame_stats(out)
    sisos = 2 * c.iterations * B * 2          # SISOs x 2 directions
    res = {"N": n, "rate": rate, "ebn0": ebn0, "B": B,
           "steps_per_siso_dir": {"phaseA": 4 * out[0] / sisos, "fixup": 4 * out[1] / sisos,
                                  "pass2": 4 * out[2] / sisos},
           "rounds_per_siso_dir": {"fixup": out[3] / sisos, "pass2": out[4] / sisos},
           "us_per_siso": {ph: round(out[i] * 0.01 / (sisos // 2), 3) for i, ph in ((5, "P"), (6, "R"), (7, "E"))}}
    if os.environ["TDEC_LIB_VARIANT"] != "frstats":   # timers-only build (TDEC_FR_STATS=2, two waves per direction)
        res = {"N": n, "rate": rate, "ebn0": ebn0, "B": B,
               "us_per_siso": res["us_per_siso"],
               "rounds_per_siso": out[2] / (sisos // 2),
               "us_per_siso_R": {"round0_phaseA": out[0] * 0.01 / (sisos // 2), "later_rounds": out[1] * 0.01 / (sisos // 2),
                                 "wave0_in_fr_round": out[3] * 0.01 / (sisos // 2),
                                 "wave0_phaseA": out[4] * 0.01 / (sisos // 2)}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
