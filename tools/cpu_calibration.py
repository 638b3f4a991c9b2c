#!/usr/bin/env python3
"""Calibrate the bench's CPU baseline (the bit-exact C restatement in oracle/)
against the reference's own numba machine code, as measured by SURVEY.md §6 in
THIS container: 12.30 ms per N=752 r=1/3 8-iteration decode on one core
(81 codewords/s), 642 codewords/s over 8 processes.

Times oracle.decode_batch on the same configuration (decode only, AWGN QPSK
LLRs at 2 dB) on 1 thread and on 8 threads, and writes
profiles/cpu_calibration.json; bench.py reports the ratio next to its
cpu_baseline.  Run here (not on the GPU box: the anchor was measured here).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from modulations_amd import tables as T  # noqa: E402

NUMBA_1CORE = 1000.0 / 12.30      # codewords/s, SURVEY.md §6 [probe]
NUMBA_8PROC = 642.0


def main():
    n, rate = 752, "1/3"
    punct = T.PUNCTURE_PATTERNS[rate]
    pm = T.puncture_matrix(punct)
    perm = T.interleaver(n)
    inv = T.inverse_interleaver(perm)
    t, G = O.trellis()
    rng = np.random.default_rng(0)
    B = 256
    info = rng.integers(0, 2, (B, 2 * n))
    coded = np.stack([O.encode(b, n, punct["period"], pm, perm, t, G) for b in info])
    n0 = 1.0 / ((1 / 3) * 2 * 10 ** 0.2)
    y = (1 - 2.0 * coded) / np.sqrt(2) + np.sqrt(n0 / 2) * rng.standard_normal(coded.shape)
    llr = (2 * np.sqrt(2) * y / n0).astype(np.float32)
    out = {}
    for threads in (1, 8):
        O.decode_batch(llr[:8], n, punct["period"], pm, 8, perm, inv, t, nthreads=threads)
        t0 = time.perf_counter()
        O.decode_batch(llr, n, punct["period"], pm, 8, perm, inv, t, nthreads=threads)
        out[f"oracle_{threads}t_cw_per_s"] = B / (time.perf_counter() - t0)
    out["numba_1core_cw_per_s"] = NUMBA_1CORE
    out["numba_8proc_cw_per_s"] = NUMBA_8PROC
    out["ratio_1core"] = out["oracle_1t_cw_per_s"] / NUMBA_1CORE
    out["ratio_8"] = out["oracle_8t_cw_per_s"] / NUMBA_8PROC
    out["config"] = "N=752 couples r=1/3, 8 iterations max-log, decode only (QPSK AWGN 2 dB LLRs), this container"
    out["host"] = open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": \t")
    json.dump(out, open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
