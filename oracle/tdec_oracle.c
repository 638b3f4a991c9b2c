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
 *   orc_siso / orc_siso64 dvb_rcs2_turbo.py:116-281 (bcjr_max_log_map; f32 / f64 channel LLRs) + build-defined log-MAP
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

/* ---------------------------------------------------------------------------
 * Build-defined log-MAP (round 3).  The reference has no current
 * log-MAP source; the historic _jacobian_log-22 was max(a,b) + log1p(exp(-|a-b|)).
 * This build keeps every log-MAP metric in BITS (base-2 logarithms: the branch
 * metrics are the reference's f64 sums with the weight 0.5 replaced by
 * 0.5*log2(e); the extrinsic goes back to nats by one f64 multiply by ln 2), so
 * the Jacobian logarithm is
 *     max*(a, b) = maxNum(a, b) + log2(1 + 2^-|a - b|),
 * evaluated with the gfx950 instructions v_exp_f32 (2^x) and v_log_f32 (log2)
 * on a quantised argument:
 *     t = |a - b| + 8          (f32: rounds |a - b| to the 2^-20 grid below 8)
 *     e = E(t) = v_exp_f32(-t) (= 2^-(|a-b|+8))
 *     w = fmaf(e, 256, 1)      (= 1 + 2^-|a-b|, one rounding)
 *     max* = maxNum(a, b) + L(w),  L = v_log_f32.
 * The +8 keeps the instruction's input on a bounded grid (t in [7.5, 48] for
 * every correction that can change a result), so its exact outputs form a
 * finite table.  E and L are faithful (within 1 ulp of the correctly rounded
 * value; tools/mb/trans_char.hip measured 2.2 % / 23 % of inputs 1 ulp off),
 * not correctly rounded, so this oracle takes them as data: orc_set_trans()
 * installs the device's exhaustive tables (captured by tdec_selftest_trans and
 * checked by the GPU tests to lie within 1 ulp of the correctly rounded values);
 * without tables the correctly rounded values are used (exp2 / log2 in f64,
 * rounded once), which is what the CPU-only accuracy tests measure.  Outside
 * the tables the hardware's behaviour is the one the tests check: NaN -> NaN,
 * E(t) <= 2^-39 for t > 48 (256 e is then absorbed: 1 + 256 e == 1, and a sum
 * that already holds a term >= 1 - 2^-23 does not change), E(+inf) = 0.
 *   lse4(x0..x3) = (Mc - 8) + L(S),  M = maxNum of the four, Mc = M + 8,
 *                  S = fmaf(E(Mc - x_i), 256, S) over i in order from S = 0
 *   (Mc - 8 is exact: M rounded to the grid of Mc, the shift every term's
 *   E(Mc - x_i) * 256 = 2^(x_i - (Mc - 8)) was taken against).
 * Branch metrics (round 4) in two halves, each an f64 sum rounded once:
 * U0 = hA + hB, U1 = hA - hB, V0 = hW + hY, V1 = hW - hY (h = 0.5 log2(e) x
 * the reference's f64 inputs); a branch of input class c = A^B and parity pair
 * wy = 2W + Y carries +-U_c + v(wy), v = {V0, V1, -V1, -V0}.
 * Recursions: each state's two parallel branches first -- their log-sum is
 * pm = v(wy) + C_c, C_c = max*(U_c, -U_c) (two max* per step) -- then
 * max*(a[p0] + pm, a[p0 + 8] + pm') over the two predecessors in table order
 * (beta: successor classes {0, 3} then {1, 2}).
 * Extrinsic: u[s][c] = alpha[s] + beta[next(s, c)] for the input classes
 * c = {0, 3}, {1, 2}; V[c][wy] = lse4 over the 4 states (in state order) whose
 * class-c branches carry the parity pair wy; X_c = lse4 over wy of
 * (v(wy) + V[c][wy]); app = {U0 + X_0, U1 + X_1, -U1 + X_1, -U0 + X_0} (inputs
 * 0..3); LpA = max*(app0, app1) - max*(app2, app3),
 * LpB = max*(app0, app2) - max*(app1, app3) (bits); Le = ((f64)Lp * ln2 - in) * sf
 * clipped to +-300.  That is the log-MAP sum (np.logaddexp over the states)
 * regrouped, so it stays within f32 rounding of log-MAP with exact f64 Jacobian
 * logarithms (tests/test_oracle_golden.py).  The HIP kernel (tdec_kernels.hip)
 * runs the same operations in the same order.
 * ------------------------------------------------------------------------- */
#define LM_C 8.0f                      /* t = |a - b| + LM_C */
#define LM_SCALE 256.0f                /* 2^LM_C */
#define LM_K 0x1.71547652b82fep-1      /* 0.5 * log2(e): the branch metrics' half weight in bits */
#define LM_LN2 0x1.62e42fefa39efp-1    /* ln 2: bits -> nats */

static const float *g_etab, *g_ltab;   /* device tables (orc_set_trans), or NULL */
static uint32_t g_elo, g_en, g_llo, g_ln;

static inline uint32_t f2u(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }

/* Install the device's exhaustive tables: etab[i] = v_exp_f32(-t) for the f32 t
 * whose bit pattern is elo + i (i < en), ltab[i] = v_log_f32(w) for the w with
 * bit pattern llo + i.  NULL tables restore the correctly rounded primitives. */
void orc_set_trans(const float *etab, uint32_t elo, uint32_t en, const float *ltab, uint32_t llo, uint32_t ln)
{
    g_etab = etab; g_elo = elo; g_en = etab ? en : 0;
    g_ltab = ltab; g_llo = llo; g_ln = ltab ? ln : 0;
}

static inline float E2neg(float t)   /* 2^-t */
{
    const uint32_t u = f2u(t);
    if (u - g_elo < g_en) return g_etab[u - g_elo];
    return (float)exp2(-(double)t);
}

static inline float L2(float w)      /* log2(w) */
{
    const uint32_t u = f2u(w);
    if (u - g_llo < g_ln) return g_ltab[u - g_llo];
    return (float)log2((double)w);
}

static inline float jac(float a, float b)   /* max* in bits */
{
    const float m = fmaxf(a, b);
    const float t = fabsf(a - b) + LM_C;
    const float w = fmaf(E2neg(t), LM_SCALE, 1.0f);
    return m + L2(w);
}

static inline float lse4(float x0, float x1, float x2, float x3)
{
    const float M = fmaxf(fmaxf(x0, x1), fmaxf(x2, x3));
    const float Mc = M + LM_C;
    float S = 0.0f;
    S = fmaf(E2neg(Mc - x0), LM_SCALE, S);
    S = fmaf(E2neg(Mc - x1), LM_SCALE, S);
    S = fmaf(E2neg(Mc - x2), LM_SCALE, S);
    S = fmaf(E2neg(Mc - x3), LM_SCALE, S);
    return (Mc - LM_C) + L2(S);   /* Mc - 8: exactly the shift the terms were taken against */
}

float orc_jac(float a, float b) { return jac(a, b); }   /* exported for the accuracy tests (bits) */
float orc_lse4(float a, float b, float c, float d) { return lse4(a, b, c, d); }

/* Channel LLRs as numba sees them: float32 arrays (every use widens them to
 * f64 first: `Lc_A[k] + La_A[k]`, `par_W * 0.5` promote) or float64 arrays
 * (numba's f64 specialisation of the same source, :135-160 / :267-268: the
 * same f64 operations on the unrounded values).  An f32 value widened is exact,
 * so one restatement over f64 inputs serves both. */
typedef struct { const void *p[4]; int f64; } lc_in;
static inline double LC(const lc_in *c, int i, int k)
{
    return c->f64 ? ((const double *)c->p[i])[k] : (double)((const float *)c->p[i])[k];
}

static void siso_exact(int N, const lc_in *lc, const double *LaA, const double *LaB, const int32_t *tables,
                       double sf, double *LeA, double *LeB);
static void siso_core(int N, const lc_in *lc, const double *LaA, const double *LaB, const int32_t *tables,
                      double sf, int algo, double *LeA, double *LeB);

/* bcjr_max_log_map, dvb_rcs2_turbo.py:116-281 (algo 0); algo 1 = the build's
 * log-MAP (above): same passes, metrics in bits, max -> max*; algo 2 = exact
 * f64 log-MAP (siso_exact, accuracy reference only). */
void orc_siso(int N, const float *LcA, const float *LcB, const float *LcW, const float *LcY,
              const double *LaA, const double *LaB, const int32_t *tables, double sf, int algo,
              double *LeA, double *LeB)
{
    const lc_in lc = {{LcA, LcB, LcW, LcY}, 0};
    if (algo == 2) siso_exact(N, &lc, LaA, LaB, tables, sf, LeA, LeB);
    else siso_core(N, &lc, LaA, LaB, tables, sf, algo, LeA, LeB);
}

/* The same with float64 channel LLRs (numba's float64 specialisation). */
void orc_siso64(int N, const double *LcA, const double *LcB, const double *LcW, const double *LcY,
                const double *LaA, const double *LaB, const int32_t *tables, double sf, int algo,
                double *LeA, double *LeB)
{
    const lc_in lc = {{LcA, LcB, LcW, LcY}, 1};
    if (algo == 2) siso_exact(N, &lc, LaA, LaB, tables, sf, LeA, LeB);
    else siso_core(N, &lc, LaA, LaB, tables, sf, algo, LeA, LeB);
}

static void siso_core(int N, const lc_in *lc, const double *LaA, const double *LaB, const int32_t *tables,
                      double sf, int algo, double *LeA, double *LeB)
{
    const int32_t *nx = tables, *ow = tables + 64, *oy = tables + 128, *ps = tables + 192, *pi = tables + 256;
    float *gamma = (float *)calloc((size_t)N * NS * 4, sizeof(float));
    float *alpha = (float *)calloc((size_t)(N + 1) * NS, sizeof(float));
    float *beta = (float *)calloc((size_t)(N + 1) * NS, sizeof(float));
    float *UV = (float *)calloc((size_t)N * 4, sizeof(float));   /* log-MAP: U0, U1, V0, V1 per k */
    const double hw = algo ? LM_K : 0.5;   /* branch-metric half weight: nats (reference) or bits */

    /* 1. gamma (:127-160): f64 sum in fixed order, stored as f32 */
    for (int k = 0; k < N; ++k) {
        double in_A = LC(lc, 0, k) + LaA[k];
        double in_B = LC(lc, 1, k) + LaB[k];
        double par_W = LC(lc, 2, k), par_Y = LC(lc, 3, k);
        if (algo) {   /* log-MAP branch halves (round 4): f64 sums rounded once */
            const double hA = in_A * hw, hB = in_B * hw, hW = par_W * hw, hY = par_Y * hw;
            UV[4 * k + 0] = (float)(hA + hB);
            UV[4 * k + 1] = (float)(hA + (-hB));
            UV[4 * k + 2] = (float)(hW + hY);
            UV[4 * k + 3] = (float)(hW + (-hY));
        }
        for (int s = 0; s < NS; ++s)
            for (int inp = 0; inp < 4; ++inp) {
                int bA = (inp >> 1) & 1, bB = inp & 1;
                int bW = ow[s * 4 + inp], bY = oy[s * 4 + inp];
                double m = 0.0;
                m += in_A * (bA == 0 ? hw : -hw);
                m += in_B * (bB == 0 ? hw : -hw);
                m += par_W * (bW == 0 ? hw : -hw);
                m += par_Y * (bY == 0 ? hw : -hw);
                gamma[((size_t)k * NS + s) * 4 + inp] = (float)m;
            }
    }
#define GAM(k, s, i) gamma[((size_t)(k) * NS + (s)) * 4 + (i)]
#define ALP(k, s) alpha[(size_t)(k) * NS + (s)]
#define BET(k, s) beta[(size_t)(k) * NS + (s)]
/* log-MAP: v(wy) = {V0, V1, -V1, -V0}; the pair of class c, parity pair wy carries
 * +-U_c + v(wy), log-sum v(wy) + C_c, C_c = max*(U_c, -U_c) */
#define LMV(k, wy) ((wy) == 0 ? UV[4 * (k) + 2] : (wy) == 1 ? UV[4 * (k) + 3] : (wy) == 2 ? -UV[4 * (k) + 3] : -UV[4 * (k) + 2])
#define LMC(k, c) jac(UV[4 * (k) + (c)], -UV[4 * (k) + (c)])
#define LMPAIR(k, s, inp) (LMV(k, 2 * ow[(s) * 4 + (inp)] + oy[(s) * 4 + (inp)]) + LMC(k, (((inp) >> 1) ^ (inp)) & 1))

    /* 2. forward, double pass (:162-197) */
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1)
            for (int s = 0; s < NS; ++s) ALP(0, s) = ALP(N, s);
        for (int k = 0; k < N; ++k) {
            for (int n = 0; n < NS; ++n) {
                float mv;
                if (algo) {
                    /* each predecessor's two parallel branches first, then the two
                     * predecessors in table order */
                    float t[2];
                    for (int q = 0; q < 2; ++q) {
                        int idx = 2 * q, p = ps[n * 4 + idx], i0 = pi[n * 4 + idx];
                        t[q] = ALP(k, p) + LMPAIR(k, p, i0);
                    }
                    mv = jac(t[0], t[1]);
                } else {
                    mv = (float)NEG_INF_VAL;
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
                float mv;
                if (algo) {
                    /* parallel pairs {0, 3} then {1, 2} (one successor each) */
                    mv = jac(BET(k + 1, nx[s * 4 + 0]) + LMPAIR(k, s, 0), BET(k + 1, nx[s * 4 + 1]) + LMPAIR(k, s, 1));
                } else {
                    mv = (float)NEG_INF_VAL;
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
        float LpA, LpB;
        if (algo) {
            /* classes c = 0 (inputs 0, 3) and 1 (inputs 1, 2): u = alpha + beta(next),
             * grouped by the branches' parity pair wy, then the branch metric per input */
            float V[2][4], X[2];
            for (int c = 0; c < 2; ++c) {
                float x[4][4];
                int cnt[4] = {0, 0, 0, 0};
                for (int s = 0; s < NS; ++s) {
                    int wy = 2 * ow[s * 4 + c] + oy[s * 4 + c];
                    x[wy][cnt[wy]++] = ALP(k, s) + BET(k + 1, nx[s * 4 + c]);
                }
                for (int wy = 0; wy < 4; ++wy) V[c][wy] = lse4(x[wy][0], x[wy][1], x[wy][2], x[wy][3]);
                /* the class's two inputs share X_c = lse4 over wy of (v(wy) + V[c][wy]) */
                X[c] = lse4(LMV(k, 0) + V[c][0], LMV(k, 1) + V[c][1], LMV(k, 2) + V[c][2], LMV(k, 3) + V[c][3]);
            }
            const float U0 = UV[4 * k], U1 = UV[4 * k + 1];
            const float app[4] = {U0 + X[0], U1 + X[1], -U1 + X[1], -U0 + X[0]};
            LpA = jac(app[0], app[1]) - jac(app[2], app[3]);
            LpB = jac(app[0], app[2]) - jac(app[1], app[3]);
        } else {
            float app[4] = {(float)NEG_INF_VAL, (float)NEG_INF_VAL, (float)NEG_INF_VAL, (float)NEG_INF_VAL};
            for (int s = 0; s < NS; ++s)
                for (int inp = 0; inp < 4; ++inp) {
                    int n = nx[s * 4 + inp];
                    float metric = ALP(k, s) + GAM(k, s, inp) + BET(k + 1, n);
                    app[inp] = maxlog_acc(app[inp], metric);
                }
            float pA0 = app[0] > app[1] ? app[0] : app[1];   /* max_star, :32-35 */
            float pA1 = app[2] > app[3] ? app[2] : app[3];
            float pB0 = app[0] > app[2] ? app[0] : app[2];
            float pB1 = app[1] > app[3] ? app[1] : app[3];
            LpA = pA0 - pA1;
            LpB = pB0 - pB1;
        }
        /* log-MAP: bits -> nats by one f64 multiply */
        double a = (algo ? (double)LpA * LM_LN2 : (double)LpA) - (LC(lc, 0, k) + LaA[k]);
        double b = (algo ? (double)LpB * LM_LN2 : (double)LpB) - (LC(lc, 1, k) + LaB[k]);
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
#undef LMV
#undef LMC
#undef LMPAIR
    free(gamma); free(alpha); free(beta); free(UV);
}

/* ------------------------------------------------------ exact log-MAP -- */
/* Accuracy reference for the build-defined log-MAP (algo 2 of orc_siso /
 * orc_decode): the same SISO structure (two passes per recursion from zero,
 * state-0 normalisation, the reference's f64 extrinsic tail) with EVERY metric
 * in f64 nats and the Jacobian logarithm max(a,b) + log1p(exp(-|a-b|)) of the
 * historic _jacobian_log-22 evaluated in f64, without the
 * f32 rounding of the branch metrics.  Not bit-compared with anything: the GPU's
 * log-MAP (bits, f32 metrics, hardware exp2 / log2) is measured against it with
 * stated tolerances (tests/test_gpu_logmap.py). */
static inline double jac64(double a, double b)
{
    if (a != a) return b;   /* maxNum: a NaN operand is dropped */
    if (b != b) return a;
    const double m = a > b ? a : b, d = fabs(a - b);
    if (d != d) return m;   /* inf - inf */
    return m + log1p(exp(-d));
}

static void siso_exact(int N, const lc_in *lc, const double *LaA, const double *LaB, const int32_t *tables,
                       double sf, double *LeA, double *LeB)
{
    const int32_t *nx = tables, *ow = tables + 64, *oy = tables + 128, *ps = tables + 192, *pi = tables + 256;
    double *gamma = (double *)calloc((size_t)N * NS * 4, sizeof(double));
    double *alpha = (double *)calloc((size_t)(N + 1) * NS, sizeof(double));
    double *beta = (double *)calloc((size_t)(N + 1) * NS, sizeof(double));
#define GAM(k, s, i) gamma[((size_t)(k) * NS + (s)) * 4 + (i)]
#define ALP(k, s) alpha[(size_t)(k) * NS + (s)]
#define BET(k, s) beta[(size_t)(k) * NS + (s)]
    for (int k = 0; k < N; ++k) {
        const double in_A = LC(lc, 0, k) + LaA[k], in_B = LC(lc, 1, k) + LaB[k];
        const double W = LC(lc, 2, k), Y = LC(lc, 3, k);
        for (int s = 0; s < NS; ++s)
            for (int inp = 0; inp < 4; ++inp) {
                int bA = (inp >> 1) & 1, bB = inp & 1, bW = ow[s * 4 + inp], bY = oy[s * 4 + inp];
                GAM(k, s, inp) = 0.5 * ((bA ? -in_A : in_A) + (bB ? -in_B : in_B) + (bW ? -W : W) + (bY ? -Y : Y));
            }
    }
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1)
            for (int s = 0; s < NS; ++s) ALP(0, s) = ALP(N, s);
        for (int k = 0; k < N; ++k) {
            for (int n = 0; n < NS; ++n) {
                double mv = -INFINITY;
                for (int idx = 0; idx < 4; ++idx) mv = jac64(mv, ALP(k, ps[n * 4 + idx]) + GAM(k, ps[n * 4 + idx], pi[n * 4 + idx]));
                ALP(k + 1, n) = mv;
            }
            const double norm = ALP(k + 1, 0);
            for (int s = 0; s < NS; ++s) ALP(k + 1, s) -= norm;
        }
    }
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1)
            for (int s = 0; s < NS; ++s) BET(N, s) = BET(0, s);
        for (int k = N - 1; k >= 0; --k) {
            for (int s = 0; s < NS; ++s) {
                double mv = -INFINITY;
                for (int inp = 0; inp < 4; ++inp) mv = jac64(mv, BET(k + 1, nx[s * 4 + inp]) + GAM(k, s, inp));
                BET(k, s) = mv;
            }
            const double norm = BET(k, 0);
            for (int s = 0; s < NS; ++s) BET(k, s) -= norm;
        }
    }
    for (int k = 0; k < N; ++k) {
        double app[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        for (int s = 0; s < NS; ++s)
            for (int inp = 0; inp < 4; ++inp) app[inp] = jac64(app[inp], ALP(k, s) + GAM(k, s, inp) + BET(k + 1, nx[s * 4 + inp]));
        double a = (jac64(app[0], app[1]) - jac64(app[2], app[3])) - (LC(lc, 0, k) + LaA[k]);
        double b = (jac64(app[0], app[2]) - jac64(app[1], app[3])) - (LC(lc, 1, k) + LaB[k]);
        a *= sf; b *= sf;
        if (a > 300.0) a = 300.0;
        if (a < -300.0) a = -300.0;
        if (b > 300.0) b = 300.0;
        if (b < -300.0) b = -300.0;
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
