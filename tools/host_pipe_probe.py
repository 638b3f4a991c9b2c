#!/usr/bin/env python3
"""Host-pointer decode throughput (DVBRCS2_Turbo.decode_batch, pageable numpy
in/out) against the chunk size of the pipelined host path (TDEC_HOST_CHUNK),
262 144 codewords; checks the bits do not depend on the chunking."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.getcwd())
from modulations_amd import dvb_rcs2_turbo as M
B = 262144
c = M.DVBRCS2_Turbo(752, "1/3")
llr = np.tile((1.0 - 2.0 * np.random.default_rng(1).integers(0, 2, (1024, c.n_coded))).astype(np.float32) * 2.0, (B // 1024, 1))
c.decode_batch(llr[:1024])
res = {}
for ch in ("262144", "131072", "65536", "32768", "16384"):
    os.environ["TDEC_HOST_CHUNK"] = ch
    c.decode_batch(llr[:65536])
    t0 = time.perf_counter(); bits = c.decode_batch(llr); dt = time.perf_counter() - t0
    res[ch] = bits
    print(f"chunk {ch}: {B / dt:,.0f} cw/s ({dt * 1e3:.0f} ms)", flush=True)
print("same:", all(np.array_equal(res["262144"], v) for v in res.values()))
