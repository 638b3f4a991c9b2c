#!/usr/bin/env python3
"""Per-wave placement and duration of one tile-decoder launch (measurement
builds with TDEC_WAVE_TIMING=1): decodes one batch with each given library,
the library appends (wave, start, end, tiles, HW_ID, XCC_ID, shader-clock start,
end) rows to $TDEC_WAVE_DUMP at tdec_destroy; then summarises waves per CU / per
SIMD against wave duration, and the shader clock the waves ran at (s_memtime
ticks over s_memrealtime's 100 MHz: the DVFS state under this kernel).

  TDEC_WAVE_DUMP=out.txt python tools/wave_dump.py lib_a.so [lib_b.so] --n 212 --mod QPSK --batch 102400
"""
import argparse
import collections
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def decode(libs, a):
    import torch
    from modulations_amd import _native, tables as T, demap as D
    from modulations_amd import dvb_rcs2_turbo as M
    from modulations_amd.workload import make_symbols
    dev = torch.device("cuda", 0)
    codec = M.DVBRCS2_Turbo(a.n, a.rate)
    B = a.batch
    _, syms, n0 = make_symbols(codec, B, a.mod, 2.0, 99, dev)
    cons = D.constellation(a.mod)
    _, div32, nve = D.demap_mode(np.complex64, cons.dtype, np.float64(n0))
    planes = torch.empty(codec.planes_bytes(B) // 4, dtype=torch.float32, device=dev)
    codec.reserve(B)
    codec.demap_planes_device(syms, cons, D.MODULATIONS[a.mod]["bps"], nve, planes, div_f32=div32)
    torch.cuda.synchronize()
    tabs = T.packed_tables(codec.next_state, codec.out_W, codec.out_Y, codec.prev_state, codec.prev_input)
    pm = T.puncture_matrix(codec.punct)
    bits = torch.empty((B, codec.k_info), dtype=torch.int32, device=dev)
    for p in libs:
        L = C.CDLL(os.path.abspath(p))
        _native._declare(L)
        h = C.c_void_p()
        assert L.tdec_create(0, a.n, codec.punct["period"], pm.ctypes.data, 8, a.algo, codec.perm.ctypes.data,
                             codec.inv_perm.ctypes.data, tabs.ctypes.data, C.byref(h)) == 0
        assert L.tdec_reserve(h, B) == 0
        for _ in range(2):   # the dump keeps the last launch
            assert L.tdec_decode_planes_dev(h, B, planes.data_ptr(), bits.data_ptr(), None, 0) == 0
            torch.cuda.synchronize()
        L.tdec_destroy(h)


def summarise(path, libs, waves):
    blocks = open(path).read().split("# launch")[1:]
    for lib, blk in zip(libs, blocks):
        rows = [list(map(int, l.split())) for l in blk.strip().splitlines()[1:]]
        rows = [r for r in rows if r[2] > 0]
        s_last = max(r[1] for r in rows)   # the last launch's waves start within ~0.1 ms of each other
        rows = [r for r in rows if r[1] >= s_last - 50000]
        t0 = min(r[1] for r in rows)
        dur = {r[0]: (r[2] - r[1]) * 1e-5 for r in rows}
        end = {r[0]: (r[2] - t0) * 1e-5 for r in rows}

        def key_cu(r):
            hw, xcc = r[4], r[5] & 0xF
            return (xcc, (hw >> 13) & 0x7, (hw >> 12) & 1, (hw >> 8) & 0xF)

        def key_simd(r):
            return key_cu(r) + (((r[4] >> 4) & 0x3),)
        per_cu = collections.Counter(key_cu(r) for r in rows)
        per_simd = collections.Counter(key_simd(r) for r in rows)
        print(f"{os.path.basename(lib)}: {len(rows)} waves on {len(per_cu)} CUs / {len(per_simd)} SIMDs; "
              f"launch {max(end.values()):.2f} ms")
        print("  waves per CU histogram:", sorted(collections.Counter(per_cu.values()).items()))
        print("  waves per SIMD histogram:", sorted(collections.Counter(per_simd.values()).items()))
        for name, kf, cnt in (("CU", key_cu, per_cu), ("SIMD", key_simd, per_simd)):
            by = collections.defaultdict(list)
            for r in rows:
                by[cnt[kf(r)]].append(dur[r[0]])
            print(f"  mean wave duration by waves on its {name}:",
                  ", ".join(f"{k}: {np.mean(v):.2f} ms (n={len(v)})" for k, v in sorted(by.items())))
        # within CUs holding 8 waves: duration by whether the SIMD has 1 or 2
        by = collections.defaultdict(list)
        for r in rows:
            by[(per_cu[key_cu(r)], per_simd[key_simd(r)])].append(dur[r[0]])
        print("  (waves on CU, waves on SIMD) -> mean ms:",
              ", ".join(f"{k}: {np.mean(v):.2f} (n={len(v)})" for k, v in sorted(by.items())))
        if all(len(r) >= 8 for r in rows):
            ghz = np.array([(r[7] - r[6]) / max(1.0, (r[2] - r[1]) * 10.0) for r in rows])
            print(f"  shader clock per wave: mean {ghz.mean():.3f} GHz, p10 {np.percentile(ghz, 10):.3f}, "
                  f"p90 {np.percentile(ghz, 90):.3f}, min {ghz.min():.3f}, max {ghz.max():.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--batch", type=int, default=102400)
    ap.add_argument("--n", type=int, default=212)
    ap.add_argument("--rate", default="1/3")
    ap.add_argument("--mod", default="QPSK")
    ap.add_argument("--algo", type=int, default=0)
    a = ap.parse_args()
    path = os.environ["TDEC_WAVE_DUMP"]
    if os.path.exists(path):
        os.remove(path)
    decode(a.libs, a)
    summarise(path, a.libs, (a.batch + 63) // 64)


if __name__ == "__main__":
    main()
