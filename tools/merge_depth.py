#!/usr/bin/env python3
"""Per-pass shader-cycle shares and merge depths of the throughput decoder
(k_turbo_decode, siso8) on a BASELINE config's device-generated inputs.  Needs
the measurement build:
  python -m modulations_amd.build --variant ptime TDEC_PASS_TIMING=1
then  python tools/merge_depth.py --n 212 --mod QPSK --batch 102400
tdec_destroy prints to stderr: F1 / F2 / B1 / B2 / epilogue shares of wave
time, and for F2 and B2 the steps each lane (and each wave's deepest lane)
ran before its pass-2 vector equalled the pass-1 one (mean, percentiles, share
of lanes that never merged)."""
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
from modulations_amd import demap as D  # noqa: E402
from modulations_amd.workload import make_symbols  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "modulations_amd", "lib", "libtdec_ptime.so"))
    ap.add_argument("--batch", type=int, default=262144)
    ap.add_argument("--n", type=int, default=752)
    ap.add_argument("--rate", default="1/3")
    ap.add_argument("--mod", default="16QAM")
    ap.add_argument("--ebn0", type=float, default=2.0)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(a.n, a.rate)
    B = a.batch
    _, syms, n0 = make_symbols(codec, B, a.mod, a.ebn0, 99, dev)
    cons = D.constellation(a.mod)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=dev)
    codec.reserve(B)
    codec.demap_planes_device(syms, cons, D.MODULATIONS[a.mod]["bps"], nve, planes, div_f32=div32)
    torch.cuda.synchronize()
    L = C.CDLL(os.path.abspath(a.lib))
    _native._declare(L)
    tabs = T.packed_tables(codec.next_state, codec.out_W, codec.out_Y, codec.prev_state, codec.prev_input)
    pm = T.puncture_matrix(codec.punct)
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    h = C.c_void_p()
    assert L.tdec_create(0, a.n, codec.punct["period"], pm.ctypes.data, 8, 0, codec.perm.ctypes.data,
                         codec.inv_perm.ctypes.data, tabs.ctypes.data, C.byref(h)) == 0, L.tdec_last_error()
    assert L.tdec_reserve(h, B) == 0
    print(f"config N={a.n} r={a.rate} {a.mod} Eb/N0={a.ebn0} dB, {B} codewords", file=sys.stderr, flush=True)
    assert L.tdec_decode_planes_dev(h, B, planes.data_ptr(), bits.data_ptr(), None, st.cuda_stream) == 0
    torch.cuda.synchronize()
    L.tdec_destroy(h)      # prints the counters of this one decode


if __name__ == "__main__":
    main()
