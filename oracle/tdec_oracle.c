/*
 * tdec_oracle.c -- CPU restatement of the reference turbo-decode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker (and the
 * "port" CPU baseline timed by bench.py).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path
 * (modulations_amd/) never links or calls it.
 *
 * Every function restates, operation for operation, the reference source in
 * /root/reference (poriya219/modulations @ 2025-12-26):
 *
 *   orc_trellis          dvb_rcs2_turbo.py:327-396  (_init_trellis)
 *   orc_interleaver      dvb_rcs2_turbo.py:311-325  (_init_interleaver; inverse = stable argsort, see below)
 *   orc_siso             dvb_rcs2_turbo.py:116-281  (bcjr_max_log_map)  + build-defined log-MAP
 *   orc_decode           dvb_rcs2_turbo.py:464-537  (DVBRCS2_Turbo.decode)
 *   orc_encode           dvb_rcs2_turbo.py:37-114, 404-462 (GF(2) helpers, _encode_component, encode)
 *   orc_demap_c64/_c128  test_sdr_with_coding.py:200-225 (compute_llr) + numpy's complex |.|
 *
 * Numerics: strict IEEE (compile with -O2 -ffp-contract=off, no -ffast-math).
 * Mixed precision exactly as numba types the reference: branch metrics summed in
 * f64 and stored f32; alpha/beta in f32; running maxima compare f32 values
 * against the f64 constant -1e9 (exactly representable in f32); extrinsic tail
 * in f64.  The pinned golden vectors in tests/golden/ (generated from the
 * reference itself by tests/golden/make_golden.py) are the check on this file.
 *
 * inv_perm: the reference uses np.argsort(perm) (unstable, host-SIMD dependent
 * tie order: SURVEY fact 4).  orc_interleaver returns the stable argsort, the
 * build's canonical pin; callers may pass any other inverse explicitly.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NS 16
#define NEG_INF_VAL (-1e9)

/* ---------------------------------------------------------------- tables -- */

/* dvb_rcs2_turbo.py:327-396.  tables layout: 5 x [16][4] int32:
 * next_state, out_W, out_Y, prev_state, prev_input. G: [4][4]. */
void orc_trellis(int32_t *tables, int32_t *G)
{
    int32_t *nx = tables, *ow = tables + 64, *oy = tables + 128, *ps = tables + 192, *pi = tables + 256;
    int counts[NS] = {0};
    for (int s = 0; s < NS; ++s) {
        int s0 = s & 1, s1 = (s >> 1) & 1, s2 = (s >> 2) & 1, s3 = (s >> 3) & 1;
        for (int inp = 0; inp < 4; ++inp) {
            int A = (inp >> 1) & 1, B = inp & 1;
            int dk = A ^ B ^ s2 ^ s3;
            int w = dk ^ s0 ^ s1 ^ s3;
            int y = dk ^ s1 ^ s2 ^ s3;
            nx[s * 4 + inp] = (s2 << 3) | (s1 << 2) | (s0 << 1) | dk;
            ow[s * 4 + inp] = w;
            oy[s * 4 + inp] = y;
        }
    }
    for (int i = 0; i < 64; ++i) { ps[i] = -1; pi[i] = -1; }
    for (int s = 0; s < NS; ++s)
        for (int inp = 0; inp < 4; ++inp) {
            int ns = nx[s * 4 + inp];
            int idx = counts[ns];
            if (idx < 4) { ps[ns * 4 + idx] = s; pi[ns * 4 + idx] = inp; counts[ns]++; }
        }
    if (G) {
        memset(G, 0, 16 * sizeof(int32_t));
        G[0 * 4 + 2] = 1; G[0 * 4 + 3] = 1; G[1 * 4 + 0] = 1; G[2 * 4 + 1] = 1; G[3 * 4 + 2] = 1;
    }
}

/* dvb_rcs2_turbo.py:311-325.  params = (P, Q0, Q1, Q2, Q3). */
void orc_interleaver(int N, const int32_t *params, int32_t *perm, int32_t *inv_stable)
{
    int64_t P = params[0], Q[3] = {params[1], params[2], params[3]}, Q3 = params[4];
    for (int i = 0; i < N; ++i) {
        int r = i % 4;
        int64_t d = r == 0 ? 0 : Q[r - 1];
        perm[i] = (int32_t)((P * (i + d + Q3 * (i / 4))) % N);
    }
    if (inv_stable) { /* stable argsort = counting sort by value, ties in index order */
        int k = 0;
        for (int v = 0; v < N; ++v)
            for (int i = 0; i < N; ++i)
                if (perm[i] == v) inv_stable[k++] = i;
    }
}

/* ------------------------------------------------------------------ SISO -- */

static inline float maxlog_acc(float acc, float t) { return t > acc ? t : acc; }

/* Build-defined log-MAP max* (SURVEY §8 a11): Jacobian logarithm
 * max(a,b) + log1p(exp(-|a-b|)) (the historic _jacobian_log-22 cut it off at
 * |a-b| > 37; here exp itself underflows to 0 past 104).  The correction is DEFINED as the fixed sequence of
 * f32 IEEE operations below -- exp(-d) = 2^-n * 2^-f from x = d*log2(e) (f = x - n
 * exact), a degree-5 polynomial for 2^-f and log1p(e) = e * Q(e) with a degree-7 Q,
 * all as fused multiply-adds
 * (fmaf is correctly rounded everywhere) -- |error| < 2.5e-7 against the real
 * function.  The HIP kernel (modulations_amd/csrc/tdec_kernels.hip, jac_corr)
 * restates it bit for bit instead of depending on two different libms. */
static inline float exp_neg(float d)   /* exp(-d), 0 <= d <= 150 */
{
    const float x = d * 0x1.715476p+0f;                     /* d * log2(e) */
    const int n = (int)x;
    const float f = x - (float)n;                             /* exact, in [0, 1) */
    float p = -0x1.f0ca8p-11f;                                /* 2^-f */
    p = fmaf(p, f, 0x1.2dd26cp-7f);
    p = fmaf(p, f, -0x1.c503aep-5f);
    p = fmaf(p, f, 0x1.ebe33ap-3f);
    p = fmaf(p, f, -0x1.62e3aap-1f);
    p = fmaf(p, f, 0x1.fffffep-1f);
    return ldexpf(p, -n);
}

static inline float log1p_01(float e)   /* log1p(e), e in [0, 1] */
{
    float q = -0x1.18f998p-7f;                                /* log1p(e) / e */
    q = fmaf(q, e, 0x1.6a33e2p-5f);
    q = fmaf(q, e, -0x1.b9c4c8p-4f);
    q = fmaf(q, e, 0x1.6ba9f2p-3f);
    q = fmaf(q, e, -0x1.f5c086p-3f);
    q = fmaf(q, e, 0x1.54bf8p-2f);
    q = fmaf(q, e, -0x1.fff95p-2f);
    q = fmaf(q, e, 0x1.fffffap-1f);
    return q * e;
}

static inline float jac_corr(float d)   /* log1p(exp(-d)), 0 <= d <= 150 */
{
    return log1p_01(exp_neg(d));
}

/* log(S) for a positive normal S: S = 2^k (1 + u), u in [0, 1) exact */
static inline float log_pos(float S)
{
    int32_t bits;
    memcpy(&bits, &S, 4);
    const int k = (bits >> 23) - 127;
    const int32_t mb = (bits & 0x7FFFFF) | 0x3F800000;
    float m;
    memcpy(&m, &mb, 4);
    return fmaf((float)k, 0x1.62e43p-1f, log1p_01(m - 1.0f));
}

/* log-MAP marginal over the 16 states (the extrinsic's app[inp], build-defined):
 * M = max_s t[s] (maxNum), S = sum over s in state order of exp(-min(M - t[s], 150)),
 * app = M + log(S).  Kernel: lse16 in tdec_kernels.hip. */
static inline float lse16(const float *t)
{
    float m = t[0];
    for (int s = 1; s < NS; ++s) m = fmaxf(m, t[s]);
    float S = 0.0f;
    for (int s = 0; s < NS; ++s) S += exp_neg(fminf(m - t[s], 150.0f));
    return m + log_pos(S);
}

/* max*(a, b) = maxNum(a, b) + log1p(exp(-min(|a - b|, 150))): the correction is
 * exactly 0 past |a - b| = 104 (exp underflows); a NaN operand is dropped. */
static inline float jac(float a, float b)
{
    return fmaxf(a, b) + jac_corr(fminf(fabsf(a - b), 150.0f));
}

float orc_jac(float a, float b) { return jac(a, b); }   /* exported for the accuracy test */

static inline float star(int algo, float a, float b)
{
    return algo ? jac(a, b) : (a > b ? a : b);   /* max_star, :32-35 */
}

/* bcjr_max_log_map, dvb_rcs2_turbo.py:116-281 (algo 0); algo 1 = log-MAP. */
void orc_siso(int N, const float *LcA, const float *LcB, const float *LcW, const float *LcY,
              const double *LaA, const double *LaB, const int32_t *tables, double sf, int algo,
              double *LeA, double *LeB)
{
    const int32_t *nx = tables, *ow = tables + 64, *oy = tables + 128, *ps = tables + 192, *pi = tables + 256;
    float *gamma = (float *)calloc((size_t)N * NS * 4, sizeof(float));
    float *alpha = (float *)calloc((size_t)(N + 1) * NS, sizeof(float));
    float *beta = (float *)calloc((size_t)(N + 1) * NS, sizeof(float));

    /* 1. gamma (:127-160): f64 sum in fixed order, stored as f32 */
    for (int k = 0; k < N; ++k) {
        double in_A = (double)LcA[k] + LaA[k];
        double in_B = (double)LcB[k] + LaB[k];
        float par_W = LcW[k], par_Y = LcY[k];
        for (int s = 0; s < NS; ++s)
            for (int inp = 0; inp < 4; ++inp) {
                int bA = (inp >> 1) & 1, bB = inp & 1;
                int bW = ow[s * 4 + inp], bY = oy[s * 4 + inp];
                double m = 0.0;
                m += in_A * (bA == 0 ? 0.5 : -0.5);
                m += in_B * (bB == 0 ? 0.5 : -0.5);
                m += (double)par_W * (bW == 0 ? 0.5 : -0.5);
                m += (double)par_Y * (bY == 0 ? 0.5 : -0.5);
                gamma[((size_t)k * NS + s) * 4 + inp] = (float)m;
            }
    }
#define GAM(k, s, i) gamma[((size_t)(k) * NS + (s)) * 4 + (i)]
#define ALP(k, s) alpha[(size_t)(k) * NS + (s)]
#define BET(k, s) beta[(size_t)(k) * NS + (s)]

    /* 2. forward, double pass (:162-197) */
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1)
            for (int s = 0; s < NS; ++s) ALP(0, s) = ALP(N, s);
        for (int k = 0; k < N; ++k) {
            for (int n = 0; n < NS; ++n) {
                float mv = (float)NEG_INF_VAL;
                if (algo) {
                    /* log-MAP (build-defined): each predecessor's two parallel
                     * branches first, max*(gamma(lower input), gamma(higher input)),
                     * then max* over the predecessors in table order */
                    for (int idx = 0; idx < 4; idx += 2) {
                        int p = ps[n * 4 + idx], i0 = pi[n * 4 + idx], i1 = pi[n * 4 + idx + 1];
                        int lo = i0 < i1 ? i0 : i1, hi = i0 < i1 ? i1 : i0;
                        mv = jac(mv, ALP(k, p) + jac(GAM(k, p, lo), GAM(k, p, hi)));
                    }
                } else {
                    for (int idx = 0; idx < 4; ++idx) {
                        int p = ps[n * 4 + idx], in = pi[n * 4 + idx];
                        float t = ALP(k, p) + GAM(k, p, in);
                        mv = maxlog_acc(mv, t);
                    }
                }
                ALP(k + 1, n) = mv;
            }
            float norm = ALP(k + 1, 0);
            for (int s = 0; s < NS; ++s) ALP(k + 1, s) -= norm;
        }
    }

    /* 3. backward, double pass (:199-230) */
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1)
            for (int s = 0; s < NS; ++s) BET(N, s) = BET(0, s);
        for (int k = N - 1; k >= 0; --k) {
            for (int s = 0; s < NS; ++s) {
                float mv = (float)NEG_INF_VAL;
                if (algo) {
                    /* log-MAP: parallel pairs {0, 3} then {1, 2} (same successor each) */
                    mv = jac(mv, BET(k + 1, nx[s * 4 + 0]) + jac(GAM(k, s, 0), GAM(k, s, 3)));
                    mv = jac(mv, BET(k + 1, nx[s * 4 + 1]) + jac(GAM(k, s, 1), GAM(k, s, 2)));
                } else {
                    for (int inp = 0; inp < 4; ++inp) {
                        int n = nx[s * 4 + inp];
                        float t = BET(k + 1, n) + GAM(k, s, inp);
                        mv = maxlog_acc(mv, t);
                    }
                }
                BET(k, s) = mv;
            }
            float norm = BET(k, 0);
            for (int s = 0; s < NS; ++s) BET(k, s) -= norm;
        }
    }

    /* 4. extrinsic (:232-281) */
    for (int k = 0; k < N; ++k) {
        float app[4] = {(float)NEG_INF_VAL, (float)NEG_INF_VAL, (float)NEG_INF_VAL, (float)NEG_INF_VAL};
        if (algo) {
            for (int inp = 0; inp < 4; ++inp) {
                float t[NS];
                for (int s = 0; s < NS; ++s) t[s] = ALP(k, s) + GAM(k, s, inp) + BET(k + 1, nx[s * 4 + inp]);
                app[inp] = lse16(t);
            }
        } else {
            for (int s = 0; s < NS; ++s)
                for (int inp = 0; inp < 4; ++inp) {
                    int n = nx[s * 4 + inp];
                    float metric = ALP(k, s) + GAM(k, s, inp) + BET(k + 1, n);
                    app[inp] = maxlog_acc(app[inp], metric);
                }
        }
        float pA0 = star(algo, app[0], app[1]);
        float pA1 = star(algo, app[2], app[3]);
        float pB0 = star(algo, app[0], app[2]);
        float pB1 = star(algo, app[1], app[3]);
        float LpA = pA0 - pA1, LpB = pB0 - pB1;
        double a = (double)LpA - ((double)LcA[k] + LaA[k]);
        double b = (double)LpB - ((double)LcB[k] + LaB[k]);
        a *= sf; b *= sf;
        const double limit = 300.0;
        if (a > limit) a = limit;
        if (a < -limit) a = -limit;
        if (b > limit) b = limit;
        if (b < -limit) b = -limit;
        LeA[k] = a; LeB[k] = b;
    }
#undef GAM
#undef ALP
#undef BET
    free(gamma); free(alpha); free(beta);
}

/* ---------------------------------------------------------------- decode -- */

/* punct: 4 rows (W1, Y1, W2, Y2) x period (<= 4), row-major [4][4]. */
int orc_depuncture(int N, int period, const uint8_t *punct, const float *llr, long n_llr, float *Lc /*[6][N]*/)
{
    long idx = 0;
    memset(Lc, 0, sizeof(float) * 6 * (size_t)N);
    for (int i = 0; i < N; ++i) {
        int p = i % period;
        if (idx + 2 > n_llr) return -1;
        Lc[0 * N + i] = llr[idx++];
        Lc[1 * N + i] = llr[idx++];
        for (int r = 0; r < 4; ++r)
            if (punct[r * 4 + p]) {
                if (idx >= n_llr) return -1;   /* IndexError in the reference loop */
                Lc[(2 + r) * N + i] = llr[idx++];
            }
    }
    return 0;
}

/* DVBRCS2_Turbo.decode, dvb_rcs2_turbo.py:464-537.  Returns 0, or -1 when the
 * LLR vector is too short (the reference raises IndexError), -2 when
 * iterations < 1 (the reference raises UnboundLocalError). */
int orc_decode(int N, int period, const uint8_t *punct, int iterations, int algo,
               const int32_t *perm, const int32_t *inv_perm, const int32_t *tables,
               const float *llr, long n_llr, int32_t *bits, double *lfinal)
{
    if (iterations < 1) return -2;
    size_t n = (size_t)N;
    float *Lc = (float *)malloc(sizeof(float) * 6 * n);
    if (orc_depuncture(N, period, punct, llr, n_llr, Lc)) { free(Lc); return -1; }
    float *LcA = Lc, *LcB = Lc + n, *W1 = Lc + 2 * n, *Y1 = Lc + 3 * n, *W2 = Lc + 4 * n, *Y2 = Lc + 5 * n;
    float *LcAi = (float *)malloc(sizeof(float) * 2 * n), *LcBi = LcAi + n;
    double *buf = (double *)calloc(8 * n, sizeof(double));
    double *LaA = buf, *LaB = buf + n, *Le1A = buf + 2 * n, *Le1B = buf + 3 * n;
    double *La2A = buf + 4 * n, *La2B = buf + 5 * n, *Le2A = buf + 6 * n, *Le2B = buf + 7 * n;
    for (int it = 0; it < iterations; ++it) {
        double sf = it < iterations - 1 ? 0.7 : 1.0;
        orc_siso(N, LcA, LcB, W1, Y1, LaA, LaB, tables, sf, algo, Le1A, Le1B);
        for (size_t k = 0; k < n; ++k) {
            La2A[k] = Le1A[perm[k]]; La2B[k] = Le1B[perm[k]];
            LcAi[k] = LcA[perm[k]]; LcBi[k] = LcB[perm[k]];
        }
        orc_siso(N, LcAi, LcBi, W2, Y2, La2A, La2B, tables, sf, algo, Le2A, Le2B);
        for (size_t k = 0; k < n; ++k) { LaA[k] = Le2A[inv_perm[k]]; LaB[k] = Le2B[inv_perm[k]]; }
    }
    for (size_t k = 0; k < n; ++k) {
        double fa = ((double)LcA[k] + LaA[k]) + Le1A[k];
        double fb = ((double)LcB[k] + LaB[k]) + Le1B[k];
        bits[2 * k] = fa < 0 ? 1 : 0;
        bits[2 * k + 1] = fb < 0 ? 1 : 0;
        if (lfinal) { lfinal[2 * k] = fa; lfinal[2 * k + 1] = fb; }
    }
    free(Lc); free(LcAi); free(buf);
    return 0;
}

/* Batched decode over B codewords (row stride llr_stride floats), OpenMP over
 * codewords: the CPU baseline.  nthreads <= 0 keeps the OpenMP default. */
int orc_decode_batch(int B, int N, int period, const uint8_t *punct, int iterations, int algo,
                     const int32_t *perm, const int32_t *inv_perm, const int32_t *tables,
                     const float *llr, long llr_stride, long n_llr, int32_t *bits, double *lfinal,
                     int nthreads)
{
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int b = 0; b < B; ++b)
        err |= -orc_decode(N, period, punct, iterations, algo, perm, inv_perm, tables,
                           llr + (size_t)b * llr_stride, n_llr, bits + (size_t)b * 2 * N,
                           lfinal ? lfinal + (size_t)b * 2 * N : NULL);
    (void)nthreads;
    return -err;
}

/* ---------------------------------------------------------------- encode -- */

static void mat_mul_gf2(const int32_t *A, const int32_t *B, int32_t *C) /* :37-48 */
{
    int32_t T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            int32_t v = 0;
            for (int k = 0; k < 4; ++k) v ^= (A[i * 4 + k] & B[k * 4 + j]);
            T[i * 4 + j] = v;
        }
    memcpy(C, T, sizeof T);
}

void orc_mat_pow_gf2(const int32_t *A, long power, int32_t *res) /* :50-61 */
{
    int32_t base[16];
    memcpy(base, A, sizeof base);
    for (int i = 0; i < 16; ++i) res[i] = (i % 5) == 0;
    while (power > 0) {
        if (power % 2 == 1) mat_mul_gf2(res, base, res);
        mat_mul_gf2(base, base, base);
        power /= 2;
    }
}

int orc_solve_circular_state_gf2(const int32_t *Gp, int Z) /* :63-114 */
{
    int32_t M[4][5];
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < 4; ++j) M[i][j] = ((i == j) + Gp[i * 4 + j]) % 2;
        M[i][4] = (Z >> i) & 1;
    }
    for (int i = 0; i < 4; ++i) {
        if (M[i][i] == 0)
            for (int k = i + 1; k < 4; ++k)
                if (M[k][i] == 1) {
                    int32_t t[5];
                    memcpy(t, M[i], sizeof t); memcpy(M[i], M[k], sizeof t); memcpy(M[k], t, sizeof t);
                    break;
                }
        if (M[i][i] == 1)
            for (int k = i + 1; k < 4; ++k)
                if (M[k][i] == 1)
                    for (int j = 0; j < 5; ++j) M[k][j] ^= M[i][j];
    }
    int32_t x[4] = {0};
    for (int i = 3; i >= 0; --i) {
        int32_t s = M[i][4];
        for (int j = i + 1; j < 4; ++j) s ^= (M[i][j] & x[j]);
        x[i] = s;
    }
    int st = 0;
    for (int i = 0; i < 4; ++i) if (x[i]) st |= 1 << i;
    return st;
}

static void encode_component(int N, const int32_t *tables, const int32_t *G, const int32_t *A,
                             const int32_t *B, int32_t *W, int32_t *Y) /* :404-429 */
{
    const int32_t *nx = tables, *ow = tables + 64, *oy = tables + 128;
    int state = 0;
    for (int i = 0; i < N; ++i) state = nx[state * 4 + ((A[i] << 1) | B[i])];
    int32_t Gp[16];
    orc_mat_pow_gf2(G, N, Gp);
    state = orc_solve_circular_state_gf2(Gp, state);
    for (int i = 0; i < N; ++i) {
        int inp = (A[i] << 1) | B[i];
        W[i] = ow[state * 4 + inp];
        Y[i] = oy[state * 4 + inp];
        state = nx[state * 4 + inp];
    }
}

/* encode, dvb_rcs2_turbo.py:431-462.  Returns the number of coded bits written
 * (which, as in the reference, can differ from n_coded for rate 2/3). */
long orc_encode(int N, int period, const uint8_t *punct, const int32_t *perm, const int32_t *tables,
                const int32_t *G, const int32_t *bits, int32_t *coded)
{
    size_t n = (size_t)N;
    int32_t *buf = (int32_t *)calloc(8 * n, sizeof(int32_t));
    int32_t *A = buf, *Bb = buf + n, *W1 = buf + 2 * n, *Y1 = buf + 3 * n;
    int32_t *Ai = buf + 4 * n, *Bi = buf + 5 * n, *W2 = buf + 6 * n, *Y2 = buf + 7 * n;
    for (size_t i = 0; i < n; ++i) { A[i] = bits[2 * i]; Bb[i] = bits[2 * i + 1]; }
    encode_component(N, tables, G, A, Bb, W1, Y1);
    for (size_t i = 0; i < n; ++i) { Ai[i] = A[perm[i]]; Bi[i] = Bb[perm[i]]; }
    encode_component(N, tables, G, Ai, Bi, W2, Y2);
    long o = 0;
    for (int i = 0; i < N; ++i) {
        int p = i % period;
        coded[o++] = A[i];
        coded[o++] = Bb[i];
        if (punct[0 * 4 + p]) coded[o++] = W1[i];
        if (punct[1 * 4 + p]) coded[o++] = Y1[i];
        if (punct[2 * 4 + p]) coded[o++] = W2[i];
        if (punct[3 * 4 + p]) coded[o++] = Y2[i];
    }
    free(buf);
    return o;
}

/* ----------------------------------------------------------------- demap -- */

/* numpy's complex |z| (umath loops_unary_complex, SIMD path, FMA hosts):
 * larger * sqrt(fma(r, r, 1)), r = smaller / larger, with its inf/NaN/zero
 * masking.  np.abs(s - constellation) in compute_llr goes through it. */
static float cabs_np_f32(float re, float im)
{
    const float inf = INFINITY;
    re = fabsf(re); im = fabsf(im);
    int re_inf = re == inf, im_inf = im == inf;
    im = re_inf ? inf : im;
    re = im_inf ? inf : re;
    int re_nn = re == re, im_nn = im == im;
    im = re_nn ? im : NAN;
    re = im_nn ? re : NAN;
    float larger = re > im ? re : im;
    float smaller = im < re ? im : re;
    int div = !(larger == 0.0f || smaller == inf);
    float ratio = div ? smaller / larger : 0.0f;
    float h = sqrtf(fmaf(ratio, ratio, 1.0f));
    return h * larger;
}

static double cabs_np_f64(double re, double im)
{
    const double inf = INFINITY;
    re = fabs(re); im = fabs(im);
    int re_inf = re == inf, im_inf = im == inf;
    im = re_inf ? inf : im;
    re = im_inf ? inf : re;
    int re_nn = re == re, im_nn = im == im;
    im = re_nn ? im : NAN;
    re = im_nn ? re : NAN;
    double larger = re > im ? re : im;
    double smaller = im < re ? im : re;
    int div = !(larger == 0.0 || smaller == inf);
    double ratio = div ? smaller / larger : 0.0;
    double h = sqrt(fma(ratio, ratio, 1.0));
    return h * larger;
}

static inline double clip30(double v) /* np.clip(llr, -30, 30), NaN propagates */
{
    if (v != v) return v;
    return v < -30.0 ? -30.0 : (v > 30.0 ? 30.0 : v);
}

/* compute_llr, test_sdr_with_coding.py:200-225, complex64 symbols.
 * constellation: M complex64 points, label i = bits MSB-first (:207-208).
 * div_f32 = 1 when noise_var is a Python float (numpy >= 2 keeps the f32
 * dtype of min_d0 - min_d1), 0 when it is an np.float64 (the call site,
 * :464-471).  Output f64 [n_sym * bps], reference sign (positive -> bit 1). */
void orc_demap_c64(const float *syms, long n_sym, const float *cons, int M, int bps,
                   double noise_var, int div_f32, double *llr)
{
    double nv = (0.005 > noise_var) ? 0.005 : noise_var;   /* Python max(noise_var, 0.005) */
    float nv32 = (float)nv;
    float d[256];
    for (long i = 0; i < n_sym; ++i) {
        float sr = syms[2 * i], si = syms[2 * i + 1];
        for (int m = 0; m < M; ++m) {
            float a = cabs_np_f32(sr - cons[2 * m], si - cons[2 * m + 1]);
            d[m] = a * a;
        }
        for (int b = 0; b < bps; ++b) {
            float m0 = INFINITY, m1 = INFINITY;
            int nan0 = 0, nan1 = 0;
            for (int m = 0; m < M; ++m) {
                int bit = (m >> (bps - 1 - b)) & 1;
                float v = d[m];
                if (bit) { if (v != v) nan1 = 1; else if (v < m1) m1 = v; }
                else     { if (v != v) nan0 = 1; else if (v < m0) m0 = v; }
            }
            if (nan0) m0 = NAN;
            if (nan1) m1 = NAN;
            float diff = m0 - m1;
            double v = div_f32 ? (double)(diff / nv32) : (double)diff / nv;
            llr[i * bps + b] = clip30(v);
        }
    }
}

/* Same, complex128 arithmetic: numpy promotes s - constellation to complex128
 * when either the symbols or the constellation are complex128 (QPSK's
 * constellation is: qpsk_mod divides complex64 by np.sqrt(2), an np.float64). */
void orc_demap_c128(const double *syms, long n_sym, const double *cons, int M, int bps,
                    double noise_var, double *llr)
{
    double nv = (0.005 > noise_var) ? 0.005 : noise_var;
    double d[256];
    for (long i = 0; i < n_sym; ++i) {
        for (int m = 0; m < M; ++m) {
            double a = cabs_np_f64(syms[2 * i] - cons[2 * m], syms[2 * i + 1] - cons[2 * m + 1]);
            d[m] = a * a;
        }
        for (int b = 0; b < bps; ++b) {
            double m0 = INFINITY, m1 = INFINITY;
            int nan0 = 0, nan1 = 0;
            for (int m = 0; m < M; ++m) {
                int bit = (m >> (bps - 1 - b)) & 1;
                double v = d[m];
                if (bit) { if (v != v) nan1 = 1; else if (v < m1) m1 = v; }
                else     { if (v != v) nan0 = 1; else if (v < m0) m0 = v; }
            }
            if (nan0) m0 = NAN;
            if (nan1) m1 = NAN;
            llr[i * bps + b] = clip30((m0 - m1) / nv);
        }
    }
}
