#!/usr/bin/env python3
"""Workload-generation kernels at bench size, for rocprofv3:
1,048,576 codewords of N = 752, r = 1/3:
  k_workload (symbols): Philox info bits -> encoder -> Gray 16QAM -> AWGN, one launch
  k_workload (encode):  tdec_encode_dev of uint8 info bits -> uint8 coded bits (the staged encoder)
  k_count_errors:       decoded rows vs the regenerated info bits
  python tools/prof_workload.py [--batch 1048576]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from modulations_amd import dvb_rcs2_turbo as M  # noqa: E402
from modulations_amd.workload import count_errors, info_bits, make_symbols  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 20)
    a = ap.parse_args()
    B = a.batch
    c = M.DVBRCS2_Turbo(752, "1/3")
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        info, syms, n0 = make_symbols(c, B, "16QAM", 2.0, 5, "cuda", want_info=False)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        bits = info_bits(c, B, 5, "cuda")
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        coded = c.encode_device(bits)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        dec = torch.zeros((B, c.k_info), dtype=torch.int32, device="cuda")
        e = count_errors(c, dec, 5)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"rep {rep}: symbols {1e3 * (t1 - t0):.1f} ms, info bits {1e3 * (t2 - t1):.1f} ms, "
              f"encode {1e3 * (t3 - t2):.1f} ms, count_errors {1e3 * (t4 - t3):.1f} ms "
              f"(mean info bit {float(e.double().mean()) / c.k_info:.4f})", flush=True)
        del info, syms, bits, coded, dec, e


if __name__ == "__main__":
    main()
