#!/usr/bin/env python3
"""CPU study of a LINEAR-DOMAIN log-MAP recursion: can a decoder
that keeps alpha / beta as f32 products of 2^metric, renormalised by a power of two
per step (no transcendental on the serial chain), meet the build's stated log-MAP
tolerance (one SISO within 1e-5 + 4 ulp_f32(M) of exact f64 log-MAP, M the block's
largest |Lc + La|)?

Model (numpy, one codeword at a time; the structure the kernel would run):
  * branch metrics in bits g = 0.5 log2(e) * (+-inA +-inB +-W +-Y) (f64, rounded
    once to f32), their exponentials E = 2^g in f32 (one v_exp per metric,
    position-parallel, off the chain);
  * alpha'[k+1][ns] = sum over the 4 branches into ns of alpha'[k][ps] * E (f32),
    then scaled by 2^-e with e the exponent of the state-0 value (exact) -- the
    linear twin of the reference's state-0 normalisation; two passes per
    recursion as the reference; beta' likewise;
  * extrinsic: app[inp] = log2(sum_s alpha'[k][s] * E[k][s][inp] * beta'[k+1][ns])
    in f32, LpA / LpB by log2-sums of the app pairs, back to nats, the
    reference's f64 tail (-in, * sf, clip +-300).
Inputs: configs[3]-like channel LLRs (8PSK-scale Gaussian, |Lc| ~ 1..8) and
a-priori values of a late turbo iteration (signs of the true bits, magnitudes
up to the +-300 clip).  Reference: the oracle's exact f64 log-MAP (algo 2).

  python tools/lm_linear_study.py [--rows 24] [--n 752]
prints per a-priori scale the fraction of positions outside the tolerance and
the largest error.  Results: profiles/r05/lm_linear_study.txt."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

K = 0.5 / np.log(2.0)   # 0.5 * log2(e)


def linear_siso(Lc, La, t, sf, shifted=False):
    nx, ow, oy, ps, pi = (t[i] for i in range(5))
    N = Lc.shape[1]
    inA = Lc[0].astype(np.float64) + La[0]
    inB = Lc[1].astype(np.float64) + La[1]
    W = Lc[2].astype(np.float64)
    Y = Lc[3].astype(np.float64)
    s = np.arange(16)[:, None]
    inp = np.arange(4)[None, :]
    bA, bB = (inp >> 1) & 1, inp & 1
    sgn = lambda b: 1.0 - 2.0 * b  # noqa: E731
    g = (K * (sgn(bA)[None] * inA[:, None, None] + sgn(bB)[None] * inB[:, None, None] +
              sgn(ow)[None] * W[:, None, None] + sgn(oy)[None] * Y[:, None, None])).astype(np.float32)   # [N,16,4]
    if shifted:   # every step's metrics against their maximum: E in (0, 1], no overflow
        g = (g - g.max(axis=(1, 2), keepdims=True)).astype(np.float32)
    with np.errstate(over="ignore"):
        E = np.exp2(g.astype(np.float64)).astype(np.float32)   # f32 2^g (inf / 0 where it over- / underflows)

    def renorm(v):
        ref = np.max(v) if shifted else v[0]   # shifted: by the largest state (a power of two), else state 0
        e = np.frexp(ref)[1] if ref > 0 and np.isfinite(ref) else 0
        return (v * np.float32(2.0 ** -e)).astype(np.float32)

    with np.errstate(all="ignore"):
        alpha = np.zeros((N + 1, 16), np.float32)
        alpha[0] = 1.0
        for pas in range(2):
            if pas:
                alpha[0] = alpha[N]
            for k in range(N):
                nv = np.zeros(16, np.float32)
                for idx in range(4):
                    nv = (nv + alpha[k][ps[:, idx]] * E[k][ps[:, idx], pi[:, idx]]).astype(np.float32)
                alpha[k + 1] = renorm(nv)
        beta = np.zeros((N + 1, 16), np.float32)
        beta[N] = 1.0
        for pas in range(2):
            if pas:
                beta[N] = beta[0]
            for k in range(N - 1, -1, -1):
                nv = np.zeros(16, np.float32)
                for i in range(4):
                    nv = (nv + beta[k + 1][nx[:, i]] * E[k][:, i]).astype(np.float32)
                beta[k] = renorm(nv)
        LeA = np.zeros(N)
        LeB = np.zeros(N)
        for k in range(N):
            app = np.array([np.sum((alpha[k] * E[k][:, i] * beta[k + 1][nx[:, i]]).astype(np.float32), dtype=np.float32)
                            for i in range(4)], np.float32)
            L = np.log2(app.astype(np.float64)).astype(np.float32)
            lA = np.logaddexp2(L[0], L[1]) - np.logaddexp2(L[2], L[3])
            lB = np.logaddexp2(L[0], L[2]) - np.logaddexp2(L[1], L[3])
            a = (float(lA) * np.log(2.0) - inA[k]) * sf
            b = (float(lB) * np.log(2.0) - inB[k]) * sf
            LeA[k] = min(max(a, -300.0), 300.0) if a == a else a
            LeB[k] = min(max(b, -300.0), 300.0) if b == b else b
    return LeA, LeB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=12)
    ap.add_argument("--n", type=int, default=752)
    a = ap.parse_args()
    t, _ = O.trellis()
    rng = np.random.default_rng(1)
    n = a.n
    print(f"N = {n}, {a.rows} rows per a-priori scale; tolerance 1e-5 + 4 ulp_f32(max |Lc + La|)")
    for shifted, la_scale in [(sh, ls) for sh in (False, True) for ls in (0.0, 5.0, 20.0, 60.0, 150.0, 300.0)]:
        bad = tot = 0
        worst = 0.0
        for r in range(a.rows):
            bits = rng.integers(0, 2, (2, n))
            Lc = ((1 - 2.0 * rng.integers(0, 2, (4, n))) * 3.0 + rng.standard_normal((4, n)) * 2.0).astype(np.float32)
            Lc[0] = ((1 - 2.0 * bits[0]) * 3.0 + rng.standard_normal(n) * 2.0).astype(np.float32)
            Lc[1] = ((1 - 2.0 * bits[1]) * 3.0 + rng.standard_normal(n) * 2.0).astype(np.float32)
            La = (1 - 2.0 * bits) * np.minimum(np.abs(rng.normal(la_scale, la_scale / 3 + 1e-9, (2, n))), 300.0)
            RA, RB = O.siso(*Lc, *La, t, 0.7, algo=2)
            LA, LB = linear_siso(Lc, La, t, 0.7, shifted)
            M = max(np.max(np.abs(Lc[0] + La[0])), np.max(np.abs(Lc[1] + La[1])))
            tol = 1e-5 + 4 * np.spacing(np.float32(M))
            err = np.maximum(np.abs(LA - RA), np.abs(LB - RB))
            err[np.isnan(err)] = np.inf
            bad += int(np.sum(err > tol))
            tot += n
            worst = max(worst, float(np.max(err)))
        print(f"{'max-shifted' if shifted else 'plain      '} a-priori scale {la_scale:6.1f}: {bad}/{tot} positions outside the tolerance ({bad / tot:.2%}), "
              f"largest error {worst:.3g} nats")


if __name__ == "__main__":
    main()
