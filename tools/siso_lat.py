#!/usr/bin/env python3
"""Per-call latency of the SISO boundary bcjr_max_log_map (dvb_rcs2_turbo.py:116-281)
at N = 48 / 212 / 752 (median of 30 calls), and of bcjr_max_log_map_batch at a few
batch sizes; TDEC_LOWLAT_MAX=0 forces the one-row-per-lane kernel for comparison."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402


def main():
    c = M.DVBRCS2_Turbo(752, "1/3")
    t = (c.next_state, c.out_W, c.out_Y, c.prev_state, c.prev_input)
    rng = np.random.default_rng(0)
    out = {"lowlat_max": os.environ.get("TDEC_LOWLAT_MAX", "default"), "single_ms": {}}
    for n in (48, 212, 752):
        Lc = [(rng.standard_normal(n) * 3).astype(np.float32) for _ in range(4)]
        La = [rng.standard_normal(n) * 5 for _ in range(2)]
        M.bcjr_max_log_map(*Lc, *La, *t, n, 0.7)
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            M.bcjr_max_log_map(*Lc, *La, *t, n, 0.7)
            ts.append(time.perf_counter() - t0)
        out["single_ms"][n] = round(float(np.median(ts)) * 1e3, 4)
        # the C call alone (staging already filled: no Python-side copies or checks)
        h = M._siso_handle(n, M._tables_key(t), 0, 0)
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            h.siso_staged(h.h, 1, 0, 0.7)
            ts.append(time.perf_counter() - t0)
        out.setdefault("c_call_ms", {})[n] = round(float(np.median(ts)) * 1e3, 4)
        # float64 channel LLRs (numba's f64 specialisation)
        Lc64 = [x.astype(np.float64) for x in Lc]
        M.bcjr_max_log_map(*Lc64, *La, *t, n, 0.7)
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            M.bcjr_max_log_map(*Lc64, *La, *t, n, 0.7)
            ts.append(time.perf_counter() - t0)
        out.setdefault("single_f64_ms", {})[n] = round(float(np.median(ts)) * 1e3, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
