#!/usr/bin/env python3
"""Interleaved in-process A/B timing of libtdec variants (guide §5.4 rule 24).

  python tools/ab.py lib/libtdec.so lib/libtdec_x.so [--batch 262144 --rounds 6]

Each variant is loaded with its own ctypes handle (separate code objects in
one process), fed the same device-resident planes, and timed round-robin with
HIP events; prints median / min ms per k_turbo_decode launch and checks that
the variants produce identical bits.

Decode time depends on where in HBM the per-wave workspace lands (a process
can come out anywhere between ~71 and ~84 ms for 262144 codewords), so each
round re-creates the handles one after the other on the same freed memory;
still run both orders before trusting a difference of a few percent.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from modulations_amd import _native, tables as T  # noqa: E402
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd.workload import make_symbols  # noqa: E402


def open_lib(path):
    L = C.CDLL(os.path.abspath(path))
    _native._declare(L)
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--n", type=int, default=752)
    ap.add_argument("--rate", default="1/3")
    ap.add_argument("--algo", type=int, default=0)
    ap.add_argument("--mod", default="16QAM")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(a.n, a.rate)
    B = a.batch
    info, syms, n0 = make_symbols(codec, B, a.mod, 2.0, 99, dev)
    from modulations_amd import demap as D
    cons = D.constellation(a.mod)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=dev)
    codec.reserve(B)
    codec.demap_planes_device(syms, cons, D.MODULATIONS[a.mod]["bps"], nve, planes, div_f32=div32)
    torch.cuda.synchronize()
    tabs = T.packed_tables(codec.next_state, codec.out_W, codec.out_Y, codec.prev_state, codec.prev_input)
    pm = T.puncture_matrix(codec.punct)
    libs = [open_lib(p) for p in a.libs]
    bits = [torch.empty((B, codec.k_info), dtype=torch.int32, device=dev) for _ in libs]
    times = [[] for _ in libs]
    st = torch.cuda.current_stream()
    # Each round creates, times and destroys one handle per library in turn, so
    # the variants run on the same freed-and-reallocated workspace memory
    # (decode time depends on where the workspace lands: see DESIGN.md §6).
    for r in range(a.rounds):
        for i, L in enumerate(libs):
            h = C.c_void_p()
            rc = L.tdec_create(0, a.n, codec.punct["period"], pm.ctypes.data, 8, a.algo, codec.perm.ctypes.data,
                               codec.inv_perm.ctypes.data, tabs.ctypes.data, C.byref(h))
            assert rc == 0, L.tdec_last_error()
            assert L.tdec_reserve(h, B) == 0
            for rep in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                assert L.tdec_decode_planes_dev(h, B, planes.data_ptr(), bits[i].data_ptr(), None, st.cuda_stream) == 0
                e1.record(st)
                torch.cuda.synchronize()
                if rep:
                    times[i].append(e0.elapsed_time(e1))
            L.tdec_destroy(h)
    for p, t, b in zip(a.libs, times, bits):
        same = torch.equal(b, bits[0])
        print(f"{os.path.basename(p):28s} median {np.median(t):8.2f} ms  min {np.min(t):8.2f} ms  "
              f"cw/s {B / (np.median(t) * 1e-3):,.0f}  same_bits={same}  rounds {' '.join(f'{x:.1f}' for x in t)}")


if __name__ == "__main__":
    main()
