#!/usr/bin/env python3
"""Golden vectors for the reference's own driver, test.py (Waveform 14: QPSK,
N = 752 couples, rate 1/2, 8 iterations, Es/N0 points, LLR scale
-(2 sqrt 2) / N0 -- the script's sign, which inverts the decoder convention).

TEST INFRASTRUCTURE ONLY, run in the build container: the reference module is
imported unmodified with the no-op numba stand-in of make_golden.py, and the
recipe of test.py:52-77 is replayed step by step (seeded numpy RNG per frame:
info bits -> reference encode -> QPSK 0 -> +1 -> complex AWGN of sigma
sqrt(N0/2) -> LLRs = Re/Im * llr_scale interleaved A0 B0 A1 B1 ... as float32 ->
reference decode).  The file holds inputs and outputs only (no code):
llr_<i>, info_<i>, bits_<i>, esn0_<i>, plus the inverse interleaver the
reference used on this host (its np.argsort(perm)).

Usage:  python tests/golden/make_golden_testpy.py   (~30 s)
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, _import_reference, make_codec  # noqa: E402


def main():
    T = _import_reference()
    codec = make_codec(T, 752, "1/2", 8)
    out = {"inv_perm": np.asarray(codec.inv_perm, np.int32)}
    i = 0
    for esn0_db in (0.5, 1.5, 2.5):
        n0 = 1.0 / 10.0 ** (esn0_db / 10.0)
        sigma = np.sqrt(n0 / 2.0)
        llr_scale = -(2.0 * np.sqrt(2.0)) / n0            # test.py's scale (sign included)
        for f in range(3):
            rng = np.random.RandomState(1000 * i + 7)
            info = rng.randint(0, 2, codec.k_info)
            coded = codec.encode(info)
            sym = ((1.0 - 2.0 * coded[0::2]) + 1j * (1.0 - 2.0 * coded[1::2])) / np.sqrt(2.0)
            rx = sym + (rng.randn(len(sym)) + 1j * rng.randn(len(sym))) * sigma
            llrs = np.zeros(len(coded), dtype=np.float32)
            llrs[0::2] = np.real(rx) * llr_scale
            llrs[1::2] = np.imag(rx) * llr_scale
            bits = codec.decode(llrs)
            out[f"llr_{i}"] = llrs
            out[f"info_{i}"] = np.asarray(info, np.int32)
            out[f"bits_{i}"] = np.asarray(bits, np.int32)
            out[f"esn0_{i}"] = np.float64(esn0_db)
            print(f"frame {i}: Es/N0 {esn0_db} dB, {int((bits != info).sum())} bit errors", flush=True)
            i += 1
    np.savez_compressed(os.path.join(OUT, "testpy.npz"), **out)


if __name__ == "__main__":
    main()
