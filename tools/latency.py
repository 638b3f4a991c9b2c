#!/usr/bin/env python3
"""Per-call latency of the host-pointer drop-in at small batches:
DVBRCS2_Turbo(N, rate).decode_batch(llr[B]) for B in 1, 4, 16, 64, 256, 1024
(median of repeated calls), and decode() called once per frame as the
reference's harness does (test.py:81).  LAT_ALGO=log-map times the log-MAP
decoder.  TDEC_LOWLAT_MAX=0 in the environment
forces the throughput (one codeword per lane) decoder for comparison."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402


def main():
    n, rate = int(sys.argv[1]) if len(sys.argv) > 1 else 752, sys.argv[2] if len(sys.argv) > 2 else "1/2"
    algo = os.environ.get("LAT_ALGO", "max-log")
    c = M.DVBRCS2_Turbo(n, rate, algo=algo)
    rng = np.random.default_rng(3)
    batches = [int(b) for b in os.environ.get("LAT_BATCHES", "1,4,16,64,256,1024").split(",")]
    nmax = max(batches + [1024])
    info = rng.integers(0, 2, (1024, c.k_info))
    llr = np.stack([(1 - 2.0 * c.encode(b)) * 2.0 for b in info[:64]])
    llr = np.tile(llr, (nmax // 64 + 1, 1))[:nmax]
    llr = (llr + rng.standard_normal(llr.shape) * 1.5).astype(np.float32)
    out = {"N": n, "rate": rate, "algo": algo, "lowlat_max": os.environ.get("TDEC_LOWLAT_MAX", "default"), "batch_ms": {}}
    for B in batches:
        c.decode_batch(llr[:B])
        ts = []
        for _ in range(7 if B < 256 else 3):
            t0 = time.perf_counter()
            c.decode_batch(llr[:B])
            ts.append(time.perf_counter() - t0)
        out["batch_ms"][B] = round(float(np.median(ts)) * 1e3, 3)
    ts = []
    for f in llr[:20]:
        t0 = time.perf_counter()
        c.decode(f)
        ts.append(time.perf_counter() - t0)
    out["decode_per_frame_ms"] = round(float(np.median(ts)) * 1e3, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
