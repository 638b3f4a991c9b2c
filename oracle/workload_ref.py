"""TEST INFRASTRUCTURE ONLY -- host restatement of the counter-based workload
generator (modulations_amd/csrc/tdec_workload.hip) used to check the device
kernels.  Not a reference algorithm: the reference draws its test data with
numpy's global RNG (turbo_test_suite.py:136); the build's generator is
Philox4x32-10 (Salmon et al. SC'11, Random123 philox4x32_R(10)) counted by the
GLOBAL codeword index so data never depends on batching or sharding.  Checked
against Random123's published known-answer vectors in tests/test_workload_host.py.
"""
from __future__ import annotations

import numpy as np

INFO_DOMAIN, NOISE_DOMAIN = 0x1AF0, 0x2B0E
_M = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over broadcastable uint32 counters; returns 4 uint32 arrays."""
    c = [np.asarray(x, np.uint64) & _M for x in (c0, c1, c2, c3)]
    c0, c1, c2, c3 = np.broadcast_arrays(*c)
    k0, k1 = np.uint64(k0) & _M, np.uint64(k1) & _M
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(0x9E3779B9)) & _M
            k1 = (k1 + np.uint64(0xBB67AE85)) & _M
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & _M, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & _M
    return [x.astype(np.uint32) for x in (c0, c1, c2, c3)]


def info_bits(cw_global, n_couples, seed):
    """uint8 [len(cw_global), 2N]: info bit j = bit j%32 of word (j%128)/32 of block j/128."""
    cw = np.asarray(cw_global, np.uint64)[:, None]
    nb = (2 * n_couples + 127) // 128
    blk = np.arange(nb, dtype=np.uint64)[None, :]
    w = philox4x32_10(cw & _M, cw >> np.uint64(32), blk, INFO_DOMAIN, seed & 0xFFFFFFFF, seed >> 32)
    words = np.stack(w, axis=-1).reshape(len(cw), nb * 4)             # [cw][block*4 + q]
    bits = (words[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1
    return bits.reshape(len(cw), nb * 128)[:, :2 * n_couples].astype(np.uint8)


def awgn(cw_global, n_sym, seed, sigma):
    """complex [len(cw), n_sym] noise, Box-Muller in float64 (the device uses f32)."""
    cw = np.asarray(cw_global, np.uint64)[:, None]
    s = np.arange(n_sym, dtype=np.uint64)[None, :]
    r = philox4x32_10(cw & _M, cw >> np.uint64(32), s >> np.uint64(1), NOISE_DOMAIN, seed & 0xFFFFFFFF, seed >> 32)
    odd = (s & np.uint64(1)).astype(bool)
    a = np.where(odd, r[2], r[0])
    b = np.where(odd, r[3], r[1])
    u1 = ((a >> 8).astype(np.float64) + 0.5) * 2.0 ** -24
    u2 = ((b >> 8).astype(np.float64) + 0.5) * 2.0 ** -24
    rad = sigma * np.sqrt(-2.0 * np.log(u1))
    return rad * np.cos(2 * np.pi * u2) + 1j * rad * np.sin(2 * np.pi * u2)
