#!/usr/bin/env python3
"""Interleaved in-process A/B timing of k_demap_planes across libtdec variants
(the bench's 16QAM workload, 1 M codewords): median ms per launch and a
bit-identity check of the planes.

  python tools/ab_demap.py lib/libtdec.so lib/libtdec_x.so [--batch 1048576 --rounds 5]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from modulations_amd import demap as D, tables as T  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd.workload import make_symbols  # noqa: E402
from tools.ab import open_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--mod", default="16QAM")
    ap.add_argument("--n", type=int, default=752)
    ap.add_argument("--rate", default="1/3")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(a.n, a.rate)
    B = a.batch
    info, syms, n0 = make_symbols(codec, B, a.mod, 2.0, 99, dev)
    # the bench's table dtype (complex128 tables demap in f64, complex64 in f32)
    cons = np.ascontiguousarray(D.constellation(a.mod))
    bps = D.MODULATIONS[a.mod]["bps"]
    f64, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    cons = np.ascontiguousarray(cons.astype(np.complex128 if f64 else np.complex64))
    tabs = T.packed_tables(codec.next_state, codec.out_W, codec.out_Y, codec.prev_state, codec.prev_input)
    pm = T.puncture_matrix(codec.punct)
    libs = [open_lib(p) for p in a.libs]
    hs = []
    for L in libs:
        L.tdec_planes_bytes.restype = C.c_size_t
        h = C.c_void_p()
        assert L.tdec_create(0, a.n, codec.punct["period"], pm.ctypes.data, 8, 0, codec.perm.ctypes.data, codec.inv_perm.ctypes.data,
                             tabs.ctypes.data, C.byref(h)) == 0
        hs.append(h)
    nb = libs[0].tdec_planes_bytes(hs[0], B)
    planes = [torch.empty(nb // 4, dtype=torch.float32, device=dev) for _ in libs]
    st = torch.cuda.current_stream()
    times = [[] for _ in libs]
    for r in range(a.rounds + 1):
        for i, (L, h) in enumerate(zip(libs, hs)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            assert L.tdec_demap_planes_dev(h, B, syms.data_ptr(), syms.shape[1], cons.ctypes.data, int(f64), len(cons), bps,
                                           float(nve), int(div32), planes[i].data_ptr(), st.cuda_stream) == 0
            e1.record(st)
            torch.cuda.synchronize()
            if r:
                times[i].append(e0.elapsed_time(e1))
    for p, t, pl in zip(a.libs, times, planes):
        print(f"{os.path.basename(p):24s} k_demap_planes median {np.median(t):7.3f} ms  min {np.min(t):7.3f}  "
              f"same_planes={torch.equal(pl, planes[0])}")
    # measurement builds (TDEC_DM_STATS=1): symbols per path over one more launch
    for p, L, h, pl in zip(a.libs, libs, hs, planes):
        try:
            fn = L.tdec_demap_stats
        except AttributeError:
            continue
        out = (C.c_ulonglong * 8)()
        fn(out)
        assert L.tdec_demap_planes_dev(h, B, syms.data_ptr(), syms.shape[1], cons.ctypes.data, int(f64), len(cons), bps,
                                       float(nve), int(div32), pl.data_ptr(), st.cuda_stream) == 0
        fn(out)
        n = max(1, out[0])
        print(f"{os.path.basename(p):24s} paths: symbols {out[0]}  gray {out[1] / n:.5f}  per-axis {out[2] / n:.5f}  "
              f"scan {out[3] / n:.5f}  sep class {int(out[4]) - 1}  div_f32 {int(div32)}")
    for L, h in zip(libs, hs):
        L.tdec_destroy(h)


if __name__ == "__main__":
    main()
