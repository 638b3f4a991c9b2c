#!/usr/bin/env python3
"""Per-call workload for rocprofv3 --kernel-trace --stats: 200 bcjr_max_log_map calls
and 50 decode() calls per frame at N = 48 / 212 / 752 (and log-MAP decode() at 752
when CALL_PROBE_LOGMAP=1), so the kernel durations of the per-call paths can be set
against their host-side call times (tools/siso_lat.py, tools/latency.py)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    t = M._std_tables()[:5]
    out = {}
    for n, rate in ((48, "1/3"), (212, "1/3"), (752, "1/2")):
        Lc = [(rng.standard_normal(n) * 3).astype(np.float32) for _ in range(4)]
        La = [rng.standard_normal(n) * 5 for _ in range(2)]
        M.bcjr_max_log_map(*Lc, *La, *t, n, 0.7)
        t0 = time.perf_counter()
        for _ in range(200):
            M.bcjr_max_log_map(*Lc, *La, *t, n, 0.7)
        out[f"siso_{n}_us"] = (time.perf_counter() - t0) / 200 * 1e6
        c = M.DVBRCS2_Turbo(n, rate, algo=os.environ.get("CALL_PROBE_ALGO", "max-log"))
        llr = ((1 - 2.0 * c.encode(rng.integers(0, 2, c.k_info))) * 2.0 + rng.standard_normal(c.n_coded) * 1.5)
        llr = llr.astype(np.float32)
        c.decode(llr)
        reps = 50 if c.algo == 0 else 3
        t0 = time.perf_counter()
        for _ in range(reps):
            c.decode(llr)
        out[f"decode_{n}_us"] = (time.perf_counter() - t0) / reps * 1e6
    print(out)


if __name__ == "__main__":
    main()
