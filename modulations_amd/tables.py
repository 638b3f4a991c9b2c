"""Host-side code tables of the DVB-RCS2 duo-binary turbo code.

Pure host logic (tiny integer tables, built once per codec).  Everything here
restates the reference module's table code:

* ``INTERLEAVER_PARAMS`` / ``PUNCTURE_PATTERNS``  -- dvb_rcs2_turbo.py:12-26
* :func:`trellis_tables`                           -- dvb_rcs2_turbo.py:327-396
* :func:`interleaver`                              -- dvb_rcs2_turbo.py:311-325
* :func:`coded_size`                               -- dvb_rcs2_turbo.py:398-402
* :func:`puncture_matrix`                          -- the per-couple pattern walk of
  dvb_rcs2_turbo.py:451-460 (encode) and :476-487 (decode), as a [4][4] uint8 mask
* GF(2) helpers / circular state                   -- dvb_rcs2_turbo.py:37-114
"""
from __future__ import annotations

import os

import numpy as np

# Interleaver parameters (reference :12-17), keyed by N in couples.
INTERLEAVER_PARAMS = {
    48: (31, 4, 2, 0, 3), 64: (41, 2, 6, 4, 1),
    212: (137, 0, 6, 4, 9), 220: (143, 4, 2, 8, 5),
    424: (277, 2, 4, 0, 7), 752: (491, 0, 8, 2, 5),
    848: (553, 4, 6, 0, 3),
}

# Puncturing patterns (reference :21-26); '1' = transmitted.
PUNCTURE_PATTERNS = {
    '1/3': {'period': 1, 'W1': [1], 'Y1': [1], 'W2': [1], 'Y2': [1]},
    '1/2': {'period': 2, 'W1': [1, 0], 'Y1': [0, 1], 'W2': [1, 0], 'Y2': [0, 1]},
    '2/3': {'period': 3, 'W1': [1, 0, 0], 'Y1': [0, 1, 0], 'W2': [0, 0, 1], 'Y2': [0, 0, 0]},
    '3/4': {'period': 4, 'W1': [1, 0, 0, 0], 'Y1': [0, 1, 0, 0], 'W2': [0, 0, 1, 0], 'Y2': [0, 0, 0, 0]},
}

N_STATES = 16


def trellis_tables():
    """16-state CRSC trellis (feedback 23, W 35, Y 27 octal), :327-396.

    Returns (next_state, out_W, out_Y, prev_state, prev_input, G) as int32
    arrays, each [16,4] (G is [4,4]).
    """
    nx = np.zeros((16, 4), np.int32)
    ow = np.zeros((16, 4), np.int32)
    oy = np.zeros((16, 4), np.int32)
    for s in range(16):
        s0, s1, s2, s3 = s & 1, (s >> 1) & 1, (s >> 2) & 1, (s >> 3) & 1
        for inp in range(4):
            a, b = (inp >> 1) & 1, inp & 1
            dk = a ^ b ^ s2 ^ s3
            ow[s, inp] = dk ^ s0 ^ s1 ^ s3
            oy[s, inp] = dk ^ s1 ^ s2 ^ s3
            nx[s, inp] = (s2 << 3) | (s1 << 2) | (s0 << 1) | dk
    G = np.zeros((4, 4), np.int32)
    G[0, 2] = G[0, 3] = G[1, 0] = G[2, 1] = G[3, 2] = 1
    ps = np.full((16, 4), -1, np.int32)
    pi = np.full((16, 4), -1, np.int32)
    cnt = np.zeros(16, int)
    for s in range(16):
        for inp in range(4):
            ns = nx[s, inp]
            if cnt[ns] < 4:
                ps[ns, cnt[ns]] = s
                pi[ns, cnt[ns]] = inp
                cnt[ns] += 1
    return nx, ow, oy, ps, pi, G


def packed_tables(next_st, out_W, out_Y, prev_st, prev_inp):
    """5 x [16][4] int32, C-contiguous: the layout the C ABI takes."""
    return np.ascontiguousarray(
        np.stack([np.asarray(t, np.int32).reshape(16, 4) for t in (next_st, out_W, out_Y, prev_st, prev_inp)]))


def interleaver(n):
    """``perm`` of :311-324.  NOT a permutation for any table N."""
    if n not in INTERLEAVER_PARAMS:
        raise ValueError(f"Block size {n} not in standard tables.")
    P, Q0, Q1, Q2, Q3 = INTERLEAVER_PARAMS[n]
    i = np.arange(n, dtype=np.int64)
    d = np.choose(i % 4, [0, Q0, Q1, Q2])
    return ((P * (i + d + Q3 * (i // 4))) % n).astype(np.int32)


def inverse_interleaver(perm, mode='stable'):
    """The decoder's de-interleaving gather, ``inv_perm`` of :325.

    The reference computes ``np.argsort(perm)``; because ``perm`` has repeated
    values the result depends on numpy's (unstable) sort and therefore on the
    host CPU's SIMD path.

    mode='stable'  -- ``np.argsort(perm, kind='stable')``: the build's canonical,
                      host-independent pin (default).
    mode='numpy'   -- exactly the reference expression evaluated on THIS host.
    mode='numpy-avx512' -- the reference expression as numpy 2.2 evaluates it on
                      an AVX-512 host (the survey's container): a pinned table
                      (data/inv_perm_numpy_avx512.npz, the ``inv_default_*``
                      golden arrays), so the reference's result on that host is
                      reproduced on any host.
    """
    perm = np.asarray(perm)
    if mode == 'stable':
        return np.argsort(perm, kind='stable').astype(np.int32)
    if mode == 'numpy':
        return np.argsort(perm).astype(np.int32)
    if mode == 'numpy-avx512':
        n = len(perm)
        if n not in INTERLEAVER_PARAMS or not np.array_equal(perm, interleaver(n)):
            raise ValueError("'numpy-avx512' is pinned for the reference interleaver of the table block sizes only")
        tab = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "inv_perm_numpy_avx512.npz"),
                      allow_pickle=False)
        return tab[f"inv_{n}"].astype(np.int32)
    raise ValueError(f"unknown inverse-interleaver mode {mode!r}")


def valid_interleaver(n):
    """A true almost-regular permutation for ``interleaver='valid-perm'`` mode
    (never used for parity): pi(i) = (P'*i + 4*Q(i mod 4)) mod N, with
    Q = (0, Q0, Q1, Q2) of the table row and P' the first odd value >= P that
    is coprime with N.  Bijective because N % 4 == 0 and P' is odd and coprime."""
    import math
    P, Q0, Q1, Q2, _ = INTERLEAVER_PARAMS[n]
    while math.gcd(P, n) != 1 or P % 2 == 0:
        P += 1
    i = np.arange(n, dtype=np.int64)
    perm = (P * i + 4 * np.choose(i % 4, [0, Q0, Q1, Q2])) % n
    assert len(np.unique(perm)) == n
    return perm.astype(np.int32)


def puncture_matrix(punct):
    """[4][4] uint8 mask, rows W1, Y1, W2, Y2; columns the pattern phase."""
    m = np.zeros((4, 4), np.uint8)
    per = punct['period']
    for r, key in enumerate(('W1', 'Y1', 'W2', 'Y2')):
        m[r, :per] = punct[key]
    return m


def coded_size(n, punct):
    """n_coded of :398-402 (what the codec advertises)."""
    per = punct['period']
    bpp = 2 * per + sum(punct['W1']) + sum(punct['Y1']) + sum(punct['W2']) + sum(punct['Y2'])
    return (n // per) * bpp


def consumed_size(n, punct):
    """How many LLRs decode()'s de-puncture loop actually reads (:476-487);
    differs from coded_size when N is not a multiple of the period."""
    per = punct['period']
    tot = 0
    for i in range(n):
        p = i % per
        tot += 2 + punct['W1'][p] + punct['Y1'][p] + punct['W2'][p] + punct['Y2'][p]
    return tot


# --------------------------------------------------------------- GF(2) ------

def max_star(a, b):
    """Max-Log approximation, :32-35."""
    return a if a > b else b


def mat_mul_gf2(A, B):
    """:37-48."""
    A = np.asarray(A, np.int32)
    B = np.asarray(B, np.int32)
    return ((A.astype(np.int64) @ B.astype(np.int64)) & 1).astype(np.int32)


def mat_pow_gf2(A, power):
    """:50-61."""
    res = np.eye(4, dtype=np.int32)
    base = np.asarray(A, np.int32).copy()
    while power > 0:
        if power % 2 == 1:
            res = mat_mul_gf2(res, base)
        base = mat_mul_gf2(base, base)
        power //= 2
    return res


def solve_circular_state_gf2(G_pow_N, Z_N):
    """:63-114 (same elimination order, same treatment of a zero pivot)."""
    M = np.zeros((4, 5), np.int32)
    M[:, :4] = (np.eye(4, dtype=np.int32) + np.asarray(G_pow_N, np.int32)) % 2
    M[:, 4] = [(Z_N >> i) & 1 for i in range(4)]
    for i in range(4):
        if M[i, i] == 0:
            for k in range(i + 1, 4):
                if M[k, i] == 1:
                    M[[i, k]] = M[[k, i]]
                    break
        if M[i, i] == 1:
            for k in range(i + 1, 4):
                if M[k, i] == 1:
                    M[k, :] ^= M[i, :]
    x = np.zeros(4, np.int32)
    for i in range(3, -1, -1):
        s = M[i, 4]
        for j in range(i + 1, 4):
            s ^= M[i, j] & x[j]
        x[i] = s
    return int(sum(1 << i for i in range(4) if x[i]))


def circular_state_table(n, G):
    """Z_N -> S_c for all 16 zero-state end states (the encoder's tail-biting
    solve, :414-417), as int32[16] for the device encoder."""
    gp = mat_pow_gf2(G, n)
    return np.array([solve_circular_state_gf2(gp, z) for z in range(16)], np.int32)
