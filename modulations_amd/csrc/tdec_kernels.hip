// tdec_kernels.hip -- gfx950 kernels of the DVB-RCS2 duo-binary turbo decoder.
//
// Design: one codeword per LANE.  The 16-state trellis is a
// compile-time constant, so a wave advances 64 independent codewords through
// the alpha/beta recursions with every state metric in VGPRs and no cross-lane
// traffic at all (no shuffles, no LDS).  Per-codeword streams live in HBM in a
// "tile" layout [tile][plane][k][64 lanes]: a wave's load of one trellis step
// is one contiguous 256 B (f32) or 512 B (f64) segment, and the interleaver
// gathers (perm[k] is the same for every codeword) stay coalesced.
//
// Numerics restate dvb_rcs2_turbo.py:116-281 operation for operation:
//   gamma: f64 sum (((±A ± B) ± W) ± Y)/2 rounded once to f32      (:127-160)
//   alpha/beta: f32 add, running max from -1e9, subtract state 0   (:162-230)
//   extrinsic: (alpha + gamma) + beta in f32, max_star, f64 tail   (:232-281)
// Compiled with -ffp-contract=off (no FMA contraction) and IEEE denormals.
// fmaxf chains are value-identical to the reference's `if t > m: m = t`
// (maxNum drops a NaN operand exactly as the strict compare does; only the
// sign of an exact zero can differ, which compares equal everywhere).
//
// The alpha metrics of the second forward pass are not stored: every W-th
// vector is checkpointed and the window is recomputed (bit-exact, the same
// operations) during the final backward pass, which fuses beta and the
// extrinsic.  HBM traffic per SISO is therefore ~4 reads of the branch inputs
// + the extrinsic write + the checkpoints.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "npmath.hip"

namespace tdec {

constexpr int NS = 16;
constexpr int WAVE = 64;
constexpr float NEG = -1.0e9f;   // NEG_INF_VAL of :125, exact in f32

// ---- trellis of _init_trellis (:327-396), as constexpr bit formulas -------
__host__ __device__ constexpr int sb(int s, int i) { return (s >> i) & 1; }
__host__ __device__ constexpr int t_dk(int s, int inp) { return ((inp >> 1) & 1) ^ (inp & 1) ^ sb(s, 2) ^ sb(s, 3); }
__host__ __device__ constexpr int t_next(int s, int inp) {
    return (sb(s, 2) << 3) | (sb(s, 1) << 2) | (sb(s, 0) << 1) | t_dk(s, inp);
}
__host__ __device__ constexpr int t_ow(int s, int inp) { return t_dk(s, inp) ^ sb(s, 0) ^ sb(s, 1) ^ sb(s, 3); }
__host__ __device__ constexpr int t_oy(int s, int inp) { return t_dk(s, inp) ^ sb(s, 1) ^ sb(s, 2) ^ sb(s, 3); }
// prev_state / prev_input in the order the reference's scan fills them
__host__ __device__ constexpr int t_prev_s(int ns, int idx) { return ((ns >> 1) & 7) | ((idx >> 1) << 3); }
__host__ __device__ constexpr int t_prev_i(int ns, int idx) {
    return ((ns & 1) ^ sb(t_prev_s(ns, idx), 2) ^ sb(t_prev_s(ns, idx), 3)) ? ((idx & 1) ? 2 : 1)
                                                                           : ((idx & 1) ? 3 : 0);
}

// ---- branch metrics ---------------------------------------------------------
// Only 16 distinct values per step: g(bA,bB,bW,bY).  g(~bits) = -g(bits)
// exactly (round-to-nearest is sign-symmetric), so 8 are stored: index
// bB*4 + bW*2 + bY with bA = 0.
// Branch metrics from the channel+a-priori sums inA = f64(Lc_A) + La_A,
// inB likewise (:135-136), and the parities (:138-139).
// log-MAP (ALGO 1) keeps its metrics in bits: the half weight is 0.5 * log2(e)
// instead of 0.5 (see the log-MAP section below).
constexpr double LM_K = 0x1.71547652b82fep-1;     // 0.5 * log2(e)
constexpr double LM_LN2 = 0x1.62e42fefa39efp-1;   // ln 2: bits -> nats
// log-MAP (ALGO 1, round 4) uses the branch metric's two halves instead:
// g = {U0, U1, V0, V1, 0...} with U0 = f32(hA + hB), U1 = f32(hA - hB),
// V0 = f32(hW + hY), V1 = f32(hW - hY) (f64 sums rounded once, weights in bits):
// a branch of input class c (A^B) and parity pair wy carries +-U_c + v(wy),
// v = {V0, V1, -V1, -V0}, so a parallel pair's log-sum is v(wy) + max*(U_c, -U_c)
// (2 max* per step instead of 8; see pair_jac).
// The parities w, y arrive as f64 here: an f32 channel LLR widened exactly (the
// reference's numba promotes f32 * 0.5 to f64), or the caller's own f64 value
// when bcjr_max_log_map is given float64 channel LLRs (numba's f64
// specialisation of the same source: every sum is then f64 from unrounded
// inputs).  The f32 overload below is the same operations.
template <int ALGO = 0>
__device__ __forceinline__ void gamma_from_sums(double inA, double inB, double w, double y, float (&g)[8]) {
    constexpr double hw = ALGO ? LM_K : 0.5;
    const double hA = inA * hw, hB = inB * hw, hW = w * hw, hY = y * hw;
    if constexpr (ALGO == 1) {
        g[0] = (float)(hA + hB);
        g[1] = (float)(hA + (-hB));
        g[2] = (float)(hW + hY);
        g[3] = (float)(hW + (-hY));
        g[4] = g[5] = g[6] = g[7] = 0.0f;
        return;
    }
    const double l1[2] = {hA + hB, hA + (-hB)};
#pragma unroll
    for (int bB = 0; bB < 2; ++bB)
#pragma unroll
        for (int bW = 0; bW < 2; ++bW) {
            const double l2 = l1[bB] + (bW ? -hW : hW);
            g[bB * 4 + bW * 2 + 0] = (float)(l2 + hY);
            g[bB * 4 + bW * 2 + 1] = (float)(l2 + (-hY));
        }
}
template <int ALGO = 0>
__device__ __forceinline__ void gamma_from_sums(double inA, double inB, float w, float y, float (&g)[8]) {
    gamma_from_sums<ALGO>(inA, inB, (double)w, (double)y, g);
}

template <int ALGO = 0>
__device__ __forceinline__ void make_gamma(float a, float b, double laA, double laB, float w, float y,
                                           float (&g)[8], double &inA, double &inB) {
    inA = (double)a + laA;
    inB = (double)b + laB;
    gamma_from_sums<ALGO>(inA, inB, w, y, g);
}

__device__ __forceinline__ float gam(const float (&g)[8], int s, int inp) {
    const int bA = (inp >> 1) & 1, bB = inp & 1, bW = t_ow(s, inp), bY = t_oy(s, inp);
    return bA == 0 ? g[bB * 4 + bW * 2 + bY] : -g[(bB ^ 1) * 4 + (bW ^ 1) * 2 + (bY ^ 1)];
}

// ---- log-MAP max* (build-defined; round 3) ----------------------
// Metrics in bits (base-2 logarithms; branch metrics weighted 0.5*log2(e), the
// extrinsic converted back to nats by one f64 multiply by ln 2), so the Jacobian
// logarithm is maxNum(a, b) + log2(1 + 2^-|a-b|), evaluated by the hardware's
// v_exp_f32 / v_log_f32 on a quantised argument:
//     t = |a - b| + 8,  w = fma(v_exp_f32(-t), 256, 1),  max* = maxNum(a, b) + v_log_f32(w)
// (7 VALU operations, two of them transcendental: 16.9 ns per wave-max* per SIMD
// against 32.4 for round 2's exp / log1p polynomials, tools/mb/jac_rate.hip).
// The +8 puts the instruction's argument on a bounded f32 grid (2^-20 below
// |a-b| = 8), so its exact outputs form a finite table: the instructions are
// faithful, not correctly rounded (tools/mb/trans_char.hip), and the oracle
// (oracle/tdec_oracle.c, which spells out the whole definition) reproduces them
// bit for bit from the device's exhaustive tables (tdec_selftest_trans).
constexpr float LM_C = 8.0f, LM_SCALE = 256.0f;   // t = |a - b| + LM_C, 2^LM_C
__device__ __forceinline__ float hw_exp2(float x) { return __builtin_amdgcn_exp2f(x); }   // v_exp_f32
__device__ __forceinline__ float hw_log2(float x) { return __builtin_amdgcn_logf(x); }    // v_log_f32

typedef float f2 __attribute__((ext_vector_type(2)));   // v_pk_add_f32 / v_pk_fma_f32 / v_pk_mul_f32: two IEEE f32 ops per lane

// (A correction log2(1 + 2^-d) from an LDS table -- {value, slope} on a 1/256 grid
// of d in [0, 24), linear interpolation: d * 256, cvt, min, fract, ds_read_b64, fma
// in place of the two transcendentals -- measured 14 % slower at configs[3]: 141.5
// vs 123.8 ms per 262 144 codewords, +23 % VALU instructions and 4.1e9 LDS reads
// with 5 bank-conflict cycles each, profiles/r06/b/, round 6.)
__device__ __forceinline__ float jac(float a, float b) {
    const float t = fabsf(a - b) + LM_C;
    const float w = fmaf(hw_exp2(-t), LM_SCALE, 1.0f);
    return fmaxf(a, b) + hw_log2(w);
}

// log2(2^x0 + 2^x1 + 2^x2 + 2^x3): the terms against Mc = max + 8, summed in
// order by fma, plus Mc - 8 (exact: the maximum rounded to Mc's grid, the shift
// the terms were taken against).
__device__ __forceinline__ float lse4(float x0, float x1, float x2, float x3) {
    const float Mc = fmaxf(fmaxf(x0, x1), fmaxf(x2, x3)) + LM_C;
    float S = hw_exp2(-(Mc - x0)) * LM_SCALE;   // = fma(e, 256, 0): exact
    S = fmaf(hw_exp2(-(Mc - x1)), LM_SCALE, S);
    S = fmaf(hw_exp2(-(Mc - x2)), LM_SCALE, S);
    S = fmaf(hw_exp2(-(Mc - x3)), LM_SCALE, S);
    return (Mc - LM_C) + hw_log2(S);
}

// The extrinsic's state groups: for input class c (0: inputs {0, 3}, 1: {1, 2},
// the same A^B and so the same successor and parity bits) the 4 states, in
// state order, whose class-c branches carry the parity pair wy = 2W + Y.
struct LmGroups {
    int s[2][4][4];
};
__host__ __device__ constexpr LmGroups make_lm_groups() {
    LmGroups G{};
    for (int c = 0; c < 2; ++c) {
        int cnt[4] = {0, 0, 0, 0};
        for (int s = 0; s < 16; ++s) {
            const int wy = 2 * t_ow(s, c) + t_oy(s, c);
            G.s[c][wy][cnt[wy]++] = s;
        }
    }
    return G;
}
constexpr LmGroups LM_GROUPS = make_lm_groups();

// ---- recursions -----------------------------------------------------------------
// max-log: the two branches of a parallel pair (inputs 0/3, or 1/2: same A^B, so
// the same next state, W and Y) leave one state for the same next state, and
// round-to-nearest is monotone, so  max(f32(m + g), f32(m + g')) == f32(m + max(g, g'))
// for every f32 m, g, g' (a NaN or -inf candidate is dropped either way: it can
// never beat the -1e9 seed).  The recursions therefore add and compare once per
// pair: pm[0][wy] = max over inputs {0, 3}, pm[1][wy] over {1, 2}, wy = 2*W + Y.
__device__ __forceinline__ void pair_max(const float (&g)[8], float (&pm)[2][4]) {
#pragma unroll
    for (int wy = 0; wy < 4; ++wy) {
        pm[0][wy] = fmaxf(g[wy], -g[3 - wy]);            // g(A0 B0 wy), g(A1 B1 wy) = -g(A0 B0 ~wy)
        pm[1][wy] = fmaxf(g[4 + wy], -g[4 + 3 - wy]);    // g(A0 B1 wy), g(A1 B0 wy) = -g(A0 B1 ~wy)
    }
}
// log-MAP's pair values (round 4): the pair of class c and parity pair wy carries
// +-U_c + v(wy), so its log-sum is v(wy) + C_c with C_c = max*(U_c, -U_c): two max*
// per step (round 3 took one per pair, eight, from the rounded full branch metrics)
__device__ __forceinline__ float lm_v(const float (&g)[8], int wy) {   // v = {V0, V1, -V1, -V0}
    return wy == 0 ? g[2] : wy == 1 ? g[3] : wy == 2 ? -g[3] : -g[2];
}
__device__ __forceinline__ void pair_jac(const float (&g)[8], float (&pm)[2][4]) {
    const float C0 = jac(g[0], -g[0]), C1 = jac(g[1], -g[1]);
#pragma unroll
    for (int wy = 0; wy < 4; ++wy) {
        pm[0][wy] = lm_v(g, wy) + C0;
        pm[1][wy] = lm_v(g, wy) + C1;
    }
}
__device__ __forceinline__ float pm_of(const float (&pm)[2][4], int s, int inp) {
    return pm[t_dk(s, inp) ^ sb(s, 2) ^ sb(s, 3)][t_ow(s, inp) * 2 + t_oy(s, inp)];
}

// The adds run two per v_pk_add_f32.  Register pairs: alpha {a[q], a[q+8]} (the two
// predecessors of a state), beta {b[2m], b[2m+1]} (the two successors of a state),
// and PM[t][wy] = {pm[t][wy], pm[1-t][3-wy]}: the two pair maxima one state's two
// branch pairs use (the other pair flips A^B, and with it W and Y).
__device__ __forceinline__ void pair_max2(const float (&g)[8], f2 (&P)[4]) {
#pragma unroll
    for (int wy = 0; wy < 4; ++wy)   // P[wy] = {pm[0][wy], pm[1][3-wy]}
        P[wy] = f2{fmaxf(g[wy], -g[3 - wy]), fmaxf(g[4 + 3 - wy], -g[4 + wy])};
}
// x + PM[t][wy], PM[t][wy] = {pm[t][wy], pm[1-t][3-wy]}: P[wy] for t = 0, and for
// t = 1 P[3-wy] with its halves swapped by the instruction's operand select
__device__ __forceinline__ f2 add_PM(f2 x, const f2 (&P)[4], int s, int inp) {
    const int t = t_dk(s, inp) ^ sb(s, 2) ^ sb(s, 3), wy = t_ow(s, inp) * 2 + t_oy(s, inp);
    if (t == 0) return x + P[wy];
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(x), "v"(P[3 - wy]));
    return r;
}

template <int ALGO> __device__ __forceinline__ void alpha_step(float (&a)[NS], const float (&g)[8]) {
    if constexpr (ALGO == 0) {
        f2 PM[4];
        pair_max2(g, PM);
        float na[NS];
#pragma unroll
        for (int ns = 0; ns < NS; ++ns) {
            const int p0 = t_prev_s(ns, 0);   // the other predecessor is p0 + 8
            const f2 t = add_PM(f2{a[p0], a[p0 + 8]}, PM, p0, t_prev_i(ns, 0));
            na[ns] = fmaxf(fmaxf(NEG, t.x), t.y);
        }
        const float norm = na[0];
#pragma unroll
        for (int s = 0; s < NS / 2; ++s) {
            const f2 v = f2{na[s], na[s + 8]} - f2{norm, norm};
            a[s] = v.x;
            a[s + 8] = v.y;
        }
        return;
    }
    // log-MAP: the parallel pair first, PM = max*(g(lower input), g(higher input)),
    // then max* over the two predecessors in table order (p0, p0 + 8)
    float pm[2][4];
    pair_jac(g, pm);
    float na[NS];
#pragma unroll
    for (int ns = 0; ns < NS; ns += 2) {
        const int p0 = t_prev_s(ns, 0), p1 = t_prev_s(ns, 2), q0 = t_prev_s(ns + 1, 0), q1 = t_prev_s(ns + 1, 2);
        const float x0 = a[p0] + pm_of(pm, p0, t_prev_i(ns, 0)), y0 = a[p1] + pm_of(pm, p1, t_prev_i(ns, 2));
        const float x1 = a[q0] + pm_of(pm, q0, t_prev_i(ns + 1, 0)), y1 = a[q1] + pm_of(pm, q1, t_prev_i(ns + 1, 2));
        na[ns] = jac(x0, y0);
        na[ns + 1] = jac(x1, y1);
    }
    const float norm = na[0];
#pragma unroll
    for (int s = 0; s < NS; ++s) a[s] = na[s] - norm;
}

template <int ALGO> __device__ __forceinline__ void beta_step(float (&b)[NS], const float (&g)[8]) {
    if constexpr (ALGO == 0) {
        f2 PM[4];
        pair_max2(g, PM);
        float nb[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int ie = (t_next(s, 0) & 1) ? 1 : 0;   // the input going to the even successor
            const int n = t_next(s, ie);
            const f2 t = add_PM(f2{b[n], b[n + 1]}, PM, s, ie);
            nb[s] = fmaxf(fmaxf(NEG, t.x), t.y);
        }
        const float norm = nb[0];
#pragma unroll
        for (int s = 0; s < NS; s += 2) {
            const f2 v = f2{nb[s], nb[s + 1]} - f2{norm, norm};
            b[s] = v.x;
            b[s + 1] = v.y;
        }
        return;
    }
    // log-MAP: pair class {0, 3} (successor next(s, 0)) first, then {1, 2}
    float pm[2][4];
    pair_jac(g, pm);
    float nb[NS];
#pragma unroll
    for (int s = 0; s < NS; s += 2) {
        const float x0 = b[t_next(s, 0)] + pm_of(pm, s, 0), y0 = b[t_next(s, 1)] + pm_of(pm, s, 1);
        const float x1 = b[t_next(s + 1, 0)] + pm_of(pm, s + 1, 0), y1 = b[t_next(s + 1, 1)] + pm_of(pm, s + 1, 1);
        nb[s] = jac(x0, y0);
        nb[s + 1] = jac(x1, y1);
    }
    const float norm = nb[0];
#pragma unroll
    for (int s = 0; s < NS; ++s) b[s] = nb[s] - norm;
}

// {x[H] + G.lo, x[H] - G.hi} (SW = 0) or {x[H] + G.hi, x[H] - G.lo} (SW = 1)
template <int H, int SW> __device__ __forceinline__ f2 pk_bcast_add_gpair(f2 x, f2 G) {
    f2 r;
    if constexpr (H == 0 && SW == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(G));
    if constexpr (H == 1 && SW == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(G));
    if constexpr (H == 0 && SW == 1) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(G));
    if constexpr (H == 1 && SW == 1) asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(G));
    return r;
}
// {t.lo + y[E], t.hi + y[E]}
template <int E> __device__ __forceinline__ f2 pk_add_bcast(f2 t, f2 y) {
    f2 r;
    if constexpr (E == 0) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0]" : "=v"(r) : "v"(t), "v"(y));
    else asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(t), "v"(y));
    return r;
}

template <int ALGO>
__device__ __forceinline__ void extrinsic(const float (&a)[NS], const float (&g)[8], const float (&b1)[NS], double inA,
                                          double inB, double sf, double &leA, double &leB) {
    float LpA, LpB;
    if constexpr (ALGO == 0) {
        float app[4];
        // (a[s] + gamma) + beta for the two inputs of a parallel pair (same next
        // state) in one lane-pair: gamma pair {g(A B wy), g(~A ~B wy)} = {g[i], -g[j]}
        // from the register pairs GP = {g0,g3}, {g1,g2}, {g4,g7}, {g5,g6}.
        const f2 GP[4] = {f2{g[0], g[3]}, f2{g[1], g[2]}, f2{g[4], g[7]}, f2{g[5], g[6]}};
#pragma unroll
        for (int i = 0; i < 4; ++i) app[i] = NEG;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const f2 A2 = f2{a[s & 7], a[(s & 7) + 8]};
#pragma unroll
            for (int T = 0; T < 2; ++T) {
                const int lo = T ? 1 : 0, hi = lo ^ 3;              // inputs {0, 3} or {1, 2}
                const int wy = t_ow(s, lo) * 2 + t_oy(s, lo);
                const int gi = 2 * T + (wy < 2 ? wy : 3 - wy);
                const int ns = t_next(s, lo);
                const f2 B2 = f2{b1[ns & ~1], b1[ns | 1]};
                f2 u;
                if (s < 8) u = wy < 2 ? pk_bcast_add_gpair<0, 0>(A2, GP[gi]) : pk_bcast_add_gpair<0, 1>(A2, GP[gi]);
                else u = wy < 2 ? pk_bcast_add_gpair<1, 0>(A2, GP[gi]) : pk_bcast_add_gpair<1, 1>(A2, GP[gi]);
                const f2 t = (ns & 1) ? pk_add_bcast<1>(u, B2) : pk_add_bcast<0>(u, B2);
                app[lo] = fmaxf(app[lo], t.x);
                app[hi] = fmaxf(app[hi], t.y);
            }
        }
        // max_star (:32-35)
        LpA = (app[0] > app[1] ? app[0] : app[1]) - (app[2] > app[3] ? app[2] : app[3]);
        LpB = (app[0] > app[2] ? app[0] : app[2]) - (app[1] > app[3] ? app[1] : app[3]);
    } else {
        // log-MAP: app[inp] = log2-sum over the 16 states of alpha + gamma + beta,
        // regrouped: u = alpha[s] + beta[next(s, c)] per input class c, summed per
        // parity pair wy over its 4 states (V), then the 4 branch metrics of the
        // input on top (the gamma of a branch depends only on the input and wy).
        // (One log-sum over the 16 states per input class instead of two levels of
        // lse4 -- 16 exp + 1 log instead of 20 + 5 -- measured 1.6 % faster at
        // configs[3], profiles/r06/d/: too little to redefine the build's log-MAP.)
        float V[2][4];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int wy = 0; wy < 4; wy += 2) {
                float x[2][4];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int st = LM_GROUPS.s[c][wy + h][i];
                        x[h][i] = a[st] + b1[t_next(st, c)];
                    }
                V[c][wy] = lse4(x[0][0], x[0][1], x[0][2], x[0][3]);
                V[c][wy + 1] = lse4(x[1][0], x[1][1], x[1][2], x[1][3]);
            }
        // app[inp] = +-U_c + X_c, X_c = lse4 over wy of (v(wy) + V[c][wy]): the two
        // inputs of a class share X_c (round 4; round 3 took one lse4 per input)
        float X[2];
#pragma unroll
        for (int c = 0; c < 2; ++c)
            X[c] = lse4(lm_v(g, 0) + V[c][0], lm_v(g, 1) + V[c][1], lm_v(g, 2) + V[c][2], lm_v(g, 3) + V[c][3]);
        const float app[4] = {g[0] + X[0], g[1] + X[1], -g[1] + X[1], -g[0] + X[0]};
        LpA = jac(app[0], app[1]) - jac(app[2], app[3]);
        LpB = jac(app[0], app[2]) - jac(app[1], app[3]);
    }
    // bits -> nats (log-MAP), then the reference's f64 tail (:262-281)
    double x = ((ALGO ? (double)LpA * LM_LN2 : (double)LpA) - inA) * sf;
    double y = ((ALGO ? (double)LpB * LM_LN2 : (double)LpB) - inB) * sf;
    x = x > 300.0 ? 300.0 : x;
    x = x < -300.0 ? -300.0 : x;
    y = y > 300.0 ? 300.0 : y;
    y = y < -300.0 ? -300.0 : y;
    leA = x;
    leB = y;
}

// Element `idx` of a wave-uniform base as SGPR base + 32-bit VGPR byte offset,
// so loads and stores use the saddr form instead of a 64-bit VGPR address.
template <class T> __device__ __forceinline__ T &at(T *base, unsigned idx) {
    return *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + idx * (unsigned)sizeof(T));
}
template <class T> __device__ __forceinline__ const T &at(const T *base, unsigned idx) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + idx * (unsigned)sizeof(T));
}

// ---- per-lane SISO --------------------------------------------------------------
// Workspace rows (P1, Le2, Le1 planes; alpha checkpoints): [k][wave][64].  A
// layout with the rows of 4 consecutive steps contiguous per wave
// ([k/4][wave][k%4][64]) was measured 1 % slower (round 2).
constexpr int WS_G = 1;
__device__ __forceinline__ unsigned wsrow(unsigned k, unsigned rs) { return k * rs; }
__host__ __device__ constexpr int rows_of(int N) { return N; }
// Raw branch inputs of one trellis step, 32 B per lane as two 16-B loads:
//   plain:      v = {Lc_A, Lc_B, Lc_W, Lc_Y} (f32), l = {La_A, La_B} (f64)
//   pre-summed: v = {-, -, Lc_W, Lc_Y},          l = {inA, inB} = f64(Lc) + La
struct Raw {
    float4 v;
    double2 l;
};

// ---- LDS-DMA staging (siso8) ----------------------------------------------------------
// global_load_lds: the load writes LDS directly, lane l's bytes at M0 + l*size,
// with no VGPR destination.  Issued by inline asm, not the builtin: the
// compiler's wait-count pass cannot tell one LDS-DMA target from another, so
// with the builtin it waits for every outstanding DMA (vmcnt(0)) before each
// new one and before each LDS read, which defeats the double buffering.  The
// asm DMA is invisible to that pass; the code waits for it explicitly
// (wait_vm<n>) before reading what it wrote.  M0 is set here and used by nothing
// else in these kernels (no builtin LDS DMA, no s_movrel, gfx9+ DS ops ignore it).
// LDS pointers are kept in the LDS address space (32-bit offsets): generic
// 64-bit pointers in the staging structs cost registers and were spilled.
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) float lds_f1;
typedef float f4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) f4v lds_f4;
typedef __attribute__((address_space(3))) d2v lds_d2;
__device__ __forceinline__ float4 ld4(const lds_f4 *p) {
    const f4v v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ double2 ld2(const lds_d2 *p) {
    const d2v v = *p;
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ unsigned lds_addr(const lds_void *l) {
    return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)l);
}
// The staging DMAs address memory as a wave-uniform 64-bit base in SGPRs plus a
// 32-bit per-lane byte offset (the instruction's saddr form) instead of a 64-bit
// per-lane address: one VGPR per address instead of a pair (the paired addresses
// of the backward passes' prologues were spilled).
__device__ __forceinline__ const void *uni_ptr(const void *p) {
    const unsigned long long u = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
    return (const void *)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ void glds16s(const void *base, unsigned off, lds_void *l) {
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr(l)), "v"(off), "s"(uni_ptr(base))
                 : "memory");
}
__device__ __forceinline__ void glds4s(const void *base, unsigned off, lds_void *l) {
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dword %1, %2" ::"s"(lds_addr(l)), "v"(off), "s"(uni_ptr(base))
                 : "memory");
}
// s_waitcnt vmcnt(n) (lgkmcnt / expcnt left open): vector-memory operations
// retire in issue order, so this retires everything but the last n issued.
template <int n> __device__ __forceinline__ void wait_vm() {
    static_assert(n >= 0 && n < 16, "vmcnt immediate");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}
__device__ __forceinline__ void wait_vm_all() { wait_vm<8>(); }

// A wave's staged half window: 4 steps x {16-B plane v, 16-B plane l} x 64 lanes.
struct LdsStage {
    lds_f4 *v;
    lds_d2 *l;
    int lane;
    lds_f4 *ck = nullptr;   // siso8: this wave's alpha-checkpoint slot [4][64] float4 (LDS-DMA)
};

// Decoder 1 in the tile layout: X = [N][64] float4 {A, B, W1, Y1} (uniform
// base), a-priori La = Le2[inv_perm[k]] ([N][64] double2, the same index for
// every lane).  The all-zero a-priori of the first iteration (:490-491) is a
// zero row read with row stride 0 (L2-resident), so the loads are the same
// straight-line code in every iteration: no branch for the compiler's
// wait-count analysis to merge pessimistically.
struct TileIn {
    const float4 *X;
    const double2 *La;
    const int *la_idx;
    int lane;
    unsigned rs;   // workspace row stride (elements between trellis steps)
    __device__ __forceinline__ Raw load(int k) const {
        Raw r;
        r.v = at(X, k * WAVE + lane);
        r.l = at(La, wsrow(la_idx[k], rs) + lane);
        return r;
    }
    template <int ALGO> __device__ __forceinline__ void gamma(const Raw &r, float (&g)[8], double &iA, double &iB) const {
        make_gamma<ALGO>(r.v.x, r.v.y, r.l.x, r.l.y, r.v.z, r.v.w, g, iA, iB);
    }
    __device__ __forceinline__ void stage(int k, const LdsStage &st, int j) const {
        glds16s(X, (unsigned)(k * WAVE + lane) * 16u, st.v + j * WAVE);
        glds16s(La, (wsrow(la_idx[k], rs) + lane) * 16u, st.l + j * WAVE);
    }
    __device__ __forceinline__ Raw staged(const LdsStage &st, int j) const {
        Raw r;
        r.v = ld4(st.v + j * WAVE + lane);
        r.l = ld2(st.l + j * WAVE + lane);
        return r;
    }
    // retire all but the last stage's 4 x (X + La) DMA operations
    __device__ __forceinline__ void wait_staged() const { wait_vm<8>(); }
};

// Decoder 2: the sums inA = f64(Lc_A[perm[k]]) + Le1_A[perm[k]] (:511-516)
// gathered from decoder 1's pre-summed output P1 (P1[j] = f64(Lc_A[j]) +
// Le1_A[j], the same f64 addition), parities from Z = [N][64] float2 {W2, Y2}.
struct TileInPre {
    const float2 *Z;
    const double2 *P;
    const int *p_idx;
    int lane;
    unsigned rs;
    __device__ __forceinline__ Raw load(int k) const {
        Raw r;
        const float2 z = at(Z, k * WAVE + lane);
        r.v = make_float4(0.0f, 0.0f, z.x, z.y);
        r.l = at(P, wsrow(p_idx[k], rs) + lane);
        return r;
    }
    template <int ALGO> __device__ __forceinline__ void gamma(const Raw &r, float (&g)[8], double &iA, double &iB) const {
        iA = r.l.x;
        iB = r.l.y;
        gamma_from_sums<ALGO>(iA, iB, r.v.z, r.v.w, g);
    }
    // {W2, Y2} as two 4-B planes inside the v slot, the gathered P1 in the l slot
    __device__ __forceinline__ void stage(int k, const LdsStage &st, int j) const {
        lds_f1 *dst = reinterpret_cast<lds_f1 *>(st.v + j * WAVE);
        const unsigned zo = (unsigned)(k * WAVE + lane) * 8u;
        glds4s(Z, zo, dst);
        glds4s(Z, zo + 4u, dst + WAVE);
        glds16s(P, (wsrow(p_idx[k], rs) + lane) * 16u, st.l + j * WAVE);
    }
    __device__ __forceinline__ Raw staged(const LdsStage &st, int j) const {
        const lds_f1 *zp = reinterpret_cast<const lds_f1 *>(st.v + j * WAVE);
        Raw r;
        r.v = make_float4(0.0f, 0.0f, zp[lane], zp[WAVE + lane]);
        r.l = ld2(st.l + j * WAVE + lane);
        return r;
    }
    __device__ __forceinline__ void wait_staged() const { wait_vm<12>(); }   // 4 x (2 x W2/Y2 + P1)
};

// Decoder 1's output: P1 = f64(Lc) + Le1 for decoder 2, and (last
// iteration) Le1 itself for the final decision (:529-530).
// P1[k] is read by decoder 2 only as P1[perm[k']]: perm is not a permutation
// (355 distinct values of 752 at N = 752), so rows outside its image are never
// read and are not written (used[k] = 0): 53 % of the P1 stream at N = 752.
// Decoder 1 also skips the extrinsic (and the alpha recompute that only feeds it)
// at those positions before the last iteration (need()).
// A discarded store goes to the wave's sink row (L2-resident) instead of being
// skipped: every position issues the same stores, so the count of memory
// operations between a load and its use is the same on every path and the
// compiler's s_waitcnt does not wait for stores it need not.  (Dropping the
// discarded stores instead -- buffer stores through a resource with num_records 0
// -- cut 16 KB of the 1.18 MB per codeword and measured neutral, the clock
// unchanged at 1.66-1.68 GHz: profiles/r06/b/, round 6.)
struct TileOutPre {
    double2 *P, *Le;   // Le may be null
    int lane;
    unsigned rs;
    const int *__restrict__ used;
    double2 *sink;     // this wave's sink row
    // Whether anything reads the extrinsic at k: decoder 2 reads only the rows
    // in perm's image, so before the last iteration (Le null) the extrinsic of the
    // other 53 % (N = 752) is dead.  Wave-uniform (scalar load).
    __device__ __forceinline__ bool need(int k) const { return Le || used[k]; }
    __device__ __forceinline__ void store(int k, double a, double b, float lcA, float lcB) const {
        // wave-uniform row selects (SGPR pairs), then the lane offset
        double2 *rp = used[k] ? &at(P, wsrow(k, rs)) : sink;
        double2 *rl = Le ? &at(Le, wsrow(k, rs)) : sink;
        at(rp, (unsigned)lane) = make_double2((double)lcA + a, (double)lcB + b);
        at(rl, (unsigned)lane) = make_double2(a, b);
    }
};

struct TileOut {
    double2 *Le;
    int lane;
    unsigned rs;
    __device__ __forceinline__ bool need(int) const { return true; }
    __device__ __forceinline__ void store(int k, double a, double b, float, float) const {
        at(Le, wsrow(k, rs) + lane) = make_double2(a, b);
    }
};

// [B][N] row layout of the bcjr_max_log_map boundary (one codeword per lane).
struct RowIn {
    const float *A, *B, *W, *Y;
    const double *LaA, *LaB;
    __device__ __forceinline__ Raw load(int k) const {
        Raw r;
        r.v = make_float4(A[k], B[k], W[k], Y[k]);
        r.l = make_double2(LaA[k], LaB[k]);
        return r;
    }
    template <int ALGO> __device__ __forceinline__ void gamma(const Raw &r, float (&g)[8], double &iA, double &iB) const {
        make_gamma<ALGO>(r.v.x, r.v.y, r.l.x, r.l.y, r.v.z, r.v.w, g, iA, iB);
    }
};

// The same rows with float64 channel LLRs (numba's f64 specialisation of
// :116-281): the sums inA = Lc_A + La_A, inB are formed at the load, in f64
// from the unrounded values (:135-136), into the l slot, and the f64 parities
// travel bit for bit in the 16 B of the v slot (W in .x/.y, Y in .z/.w).  The
// siso<> code hands v.x / v.y only to the output's store, which RowOut ignores.
struct RowIn64 {
    const double *A, *B, *W, *Y;
    const double *LaA, *LaB;
    __device__ __forceinline__ Raw load(int k) const {
        Raw r;
        const double w = W[k], y = Y[k];
        r.v = make_float4(__int_as_float(__double2loint(w)), __int_as_float(__double2hiint(w)),
                          __int_as_float(__double2loint(y)), __int_as_float(__double2hiint(y)));
        r.l = make_double2(A[k] + LaA[k], B[k] + LaB[k]);
        return r;
    }
    template <int ALGO> __device__ __forceinline__ void gamma(const Raw &r, float (&g)[8], double &iA, double &iB) const {
        iA = r.l.x;
        iB = r.l.y;
        const double w = __hiloint2double(__float_as_int(r.v.y), __float_as_int(r.v.x));
        const double y = __hiloint2double(__float_as_int(r.v.w), __float_as_int(r.v.z));
        gamma_from_sums<ALGO>(iA, iB, w, y, g);
    }
};

struct RowOut {
    double *A, *B;
    bool active;
    __device__ __forceinline__ bool need(int) const { return true; }
    __device__ __forceinline__ void store(int k, double a, double b, float, float) const {
        if (active) {
            A[k] = a;
            B[k] = b;
        }
    }
};

// Stored element order of a state vector: alpha vectors (ALPHA) in their register
// pairs {a[q], a[q+8]}, so float4 #c = {a[2c], a[2c+8], a[2c+1], a[2c+9]}; beta
// vectors in natural order (their pairs {b[2m], b[2m+1]} are already adjacent).
template <bool ALPHA> __device__ __forceinline__ constexpr int vec_elem(int c, int e) {
    return ALPHA ? 2 * c + (e >> 1) + 8 * (e & 1) : 4 * c + e;
}

// c: slot base of the calling wave, cs: elements between consecutive float4 slots
template <bool ALPHA>
__device__ __forceinline__ void load_vec(float (&x)[NS], const float4 *c, unsigned cs, unsigned base, int lane) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = at(c, (base + q) * cs + lane);
        x[vec_elem<ALPHA>(q, 0)] = v.x;
        x[vec_elem<ALPHA>(q, 1)] = v.y;
        x[vec_elem<ALPHA>(q, 2)] = v.z;
        x[vec_elem<ALPHA>(q, 3)] = v.w;
    }
}

// This lane's vector equals the stored one (IEEE ==).  No short-circuit: with
// `&&` the compiler issued the four loads one after another, each behind the
// previous compare (four round trips per merge check instead of one; measured
// the same speed, r02ap_nsc.log: the other wave hides them).
template <bool ALPHA>
__device__ __forceinline__ bool lane_equal(const float (&x)[NS], const float4 *c, unsigned cs, unsigned base, int lane) {
    bool eq = true;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = at(c, (base + q) * cs + lane);
        eq &= (x[vec_elem<ALPHA>(q, 0)] == v.x) & (x[vec_elem<ALPHA>(q, 1)] == v.y) &
              (x[vec_elem<ALPHA>(q, 2)] == v.z) & (x[vec_elem<ALPHA>(q, 3)] == v.w);
    }
    return eq;
}

// Two state vectors are equal (IEEE ==, no short-circuit: one compare chain).
__device__ __forceinline__ bool vec_equal(const float (&x)[NS], const float (&y)[NS]) {
    bool eq = true;
#pragma unroll
    for (int s = 0; s < NS; ++s) eq &= x[s] == y[s];
    return eq;
}

template <bool ALPHA>
__device__ __forceinline__ void store_vec(float4 *c, unsigned cs, unsigned base, int lane, const float (&x)[NS]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
        at(c, (base + q) * cs + lane) = make_float4(x[vec_elem<ALPHA>(q, 0)], x[vec_elem<ALPHA>(q, 1)],
                                                    x[vec_elem<ALPHA>(q, 2)], x[vec_elem<ALPHA>(q, 3)]);
}

// Window of the backward sweep fused with the extrinsic (:220-281): steps
// k0+W-1 .. k0 with beta entering at position k0+W.  alpha[k] of the second
// forward pass is recomputed from the window checkpoint (the same f32
// operations, so bit-exact): holding all W alpha vectors of a window costs
// 16*W VGPRs, recomputing costs W(W-1)/2 extra steps of VALU, which this
// HBM-bound kernel has to spare.
// `raw` / `an` hold this window's inputs / alpha checkpoint on entry and the
// next (lower) window's on exit.  Both are loaded at the START of the window,
// before its extrinsic stores: vmcnt retires in issue order, so waiting for a
// load issued after a store waits for the store too.  The loads are
// unconditional (the last window re-loads its own rows), so the number of
// memory operations issued after them is the same on every path and the
// compiler's wait counts stay exact.
template <int ALGO, int W, bool RAG, class In, class Out>
__device__ __forceinline__ void back_window(const In &in, const Out &out, int k0, int len, Raw (&raw)[W],
                                            float (&an)[NS], float (&b)[NS], const float4 *ck, unsigned cs, int lane,
                                            int N, double sf) {
    // len = steps in this window (W except for a ragged top window when W does not divide N)
    float gw[W][8], lcA[W], lcB[W];
    double iAw[W], iBw[W];
#pragma unroll
    for (int j = 0; j < W; ++j) {
        in.template gamma<ALGO>(raw[j], gw[j], iAw[j], iBw[j]);
        lcA[j] = raw[j].v.x;
        lcB[j] = raw[j].v.y;
    }
    float a0[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) a0[s] = an[s];
    {
        const int kn = k0 >= W ? k0 - W : 0;
#pragma unroll
        for (int j = 0; j < W; ++j) raw[j] = in.load(RAG ? min(kn + j, N - 1) : kn + j);
        load_vec<true>(an, ck, cs, (kn / W) * 4, lane);
    }
    // alpha at the window midpoint (computed once) halves the recompute: positions
    // >= W/2 start from it, positions < W/2 from the checkpoint (log-MAP too since
    // its recursions combine branch pairs first: -5 % time, 68 instead of 270 B of
    // scratch per lane).  Skipping it where the positions it feeds are dead
    // measured neutral (log-MAP) or slower (max-log, more spills): it always runs.
    constexpr int H = W / 2;
    float am[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) am[s] = a0[s];
#pragma unroll
    for (int i = 0; i < H; ++i) alpha_step<ALGO>(am, gw[i]);
#pragma unroll
    for (int j = W - 1; j >= 0; --j) {
        if (RAG && j >= len) continue;       // wave-uniform
        __builtin_amdgcn_sched_barrier(0);   // keep the window positions from being interleaved
        const int from = j >= H ? H : 0;
        double leA = 0.0, leB = 0.0;
        if (out.need(k0 + j)) {
            float aj[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                aj[s] = j >= H ? am[s] : a0[s];
                asm volatile("" : "+v"(aj[s]));   // opaque copy: stops CSE from re-materialising the window
            }
#pragma unroll
            for (int i = from; i < j; ++i) alpha_step<ALGO>(aj, gw[i]);
            extrinsic<ALGO>(aj, gw[j], b, iAw[j], iBw[j], sf, leA, leB);
        }
        out.store(k0 + j, leA, leB, lcA[j], lcB[j]);
        beta_step<ALGO>(b, gw[j]);
    }
}

// bcjr_max_log_map (:116-281) for the calling lane's codeword, 64 lanes at once.
//
// The reference runs each recursion twice (a convergence pass from zero, then
// the pass it uses, started from the first pass's end state).  The two passes
// apply the same deterministic f32 map to the same branch metrics, so once a
// pass-2 state vector equals the pass-1 vector at the same step (IEEE ==),
// every later one does too.  They merge after a few dozen steps (measured:
// median 40, worst 122 of 752 at 2 dB), so pass 2 is run only until it has
// merged in every lane of the wave:
//   F1  alpha from 0, checkpoint alpha1 every W steps                  (:165-179)
//   F2  alpha from alpha1[N] (:182-183), overwrite checkpoints until
//       alpha2 == alpha1 at a checkpoint; the rest are alpha2's        (:186-197)
//   B1  beta from 0 (:203-213) fused with a provisional extrinsic from
//       alpha2 and beta1; beta1 kept at every RSTEP-th of the first
//       RING*RSTEP window starts
//   B2  beta from beta1[0] (:216-230), recomputing the extrinsic until
//       beta2 == beta1 at a kept window start; below that the provisional
//       values are exact (a pass that has not merged by then runs to the end).
// ck: alpha checkpoints [ceil(N/W)][4][64] float4; ring: beta1 [RING][4][64].
// Any N >= 1: only the top window can be short, every guard is wave-uniform.
// F1 of a SISO: alpha from a (zero) over all N steps, checkpoint every W steps,
// inputs software-pipelined one group of FG steps ahead.  A deeper group than
// W (FG = 8 at W = 4) measured no faster (round 2): F1's waits are already
// covered, it is the backward windows that expose latency.  log-MAP: one
// checkpoint interval per group (its steps are ~10x larger, and the kernel's
// instruction footprint, not load latency, is what costs).
constexpr int FG_ML = 4, FG_LM = 2;
// STORE = false: the recursion alone (log-MAP's F1, whose checkpoints F2 would
// overwrite almost everywhere, see siso<>).
template <int ALGO, int W, bool RAG, bool STORE = true, class In>
__device__ __forceinline__ void f1_pass(const In &in, int N, float4 *ck, unsigned cs, int lane, float (&a)[NS]) {
    constexpr int FGW = ALGO ? FG_LM : FG_ML;
    constexpr int FG = FGW > W ? FGW : W;   // a multiple of W
    static_assert(FG % W == 0, "FG must be a multiple of W");
    // steps past N exist only when W does not divide N (RAG) or FG > W
    const bool tail = RAG || (FG > W && N % FG != 0);
    Raw raw[FG];
#pragma unroll
    for (int j = 0; j < FG; ++j) raw[j] = in.load(tail ? min(j, N - 1) : j);
    for (int k0 = 0; k0 < N; k0 += FG) {
        float g[FG][8];
#pragma unroll
        for (int j = 0; j < FG; ++j) {
            if (tail && k0 + j >= N) continue;   // wave-uniform
            double iA, iB;
            in.template gamma<ALGO>(raw[j], g[j], iA, iB);
        }
        if (k0 + FG < N) {
#pragma unroll
            for (int j = 0; j < FG; ++j) raw[j] = in.load(tail ? min(k0 + FG + j, N - 1) : k0 + FG + j);
        }
#pragma unroll
        for (int j = 0; j < FG; ++j) {
            if (tail && k0 + j >= N) continue;
            if (STORE && j % W == 0) store_vec<true>(ck, cs, ((k0 + j) / W) * 4, lane, a);
            alpha_step<ALGO>(a, g[j]);
        }
    }
}

// B1 of log-MAP as a plain beta recursion (no extrinsic, no stores), then B2
// over the whole block with the extrinsic.  log-MAP's second passes merge with
// the first late (8PSK r=1/2 at 2 dB, oracle: per 64-codeword wave the last
// lane merges after 83 % (F2) / 89 % (B2) of N, median lane 27 %; max-log: 29 %),
// so the provisional extrinsic of B1 is recomputed almost everywhere anyway:
// one beta-only pass + one full pass does less work than two extrinsic passes.
// log-MAP's F1 likewise: alpha1 without checkpoints, then F2 over the whole block
// storing every checkpoint (no merge test): fewer bytes (F2 would rewrite 83 % of
// the checkpoints after reading them for the test) for 17 % more F2 steps.
template <int ALGO, bool RAG, class In>
__device__ __forceinline__ void b1_pass(const In &in, int N, float (&b)[NS]) {
    constexpr int FG = ALGO ? FG_LM : FG_ML;
    Raw raw[FG];
    // groups [k1 - FG, k1) from the top; the lowest may be short (wave-uniform guards)
#pragma unroll
    for (int j = 0; j < FG; ++j) raw[j] = in.load(max(N - FG + j, 0));
    for (int k1 = N; k1 > 0; k1 -= FG) {
        float g[FG][8];
#pragma unroll
        for (int j = 0; j < FG; ++j) {
            if (k1 - FG + j < 0) continue;   // wave-uniform
            double iA, iB;
            in.template gamma<ALGO>(raw[j], g[j], iA, iB);
        }
        if (k1 - FG > 0) {
#pragma unroll
            for (int j = 0; j < FG; ++j) raw[j] = in.load(max(k1 - 2 * FG + j, 0));
        }
#pragma unroll
        for (int j = FG - 1; j >= 0; --j)
            if (k1 - FG + j >= 0) beta_step<ALGO>(b, g[j]);
    }
}

constexpr int RING = 16;   // beta1 kept at RING window starts 16 steps apart: the top 256 steps (merge: median 40, max 122)
__host__ __device__ constexpr int rstep_of(int w) { return w >= 16 ? 1 : 16 / w; }

// Issue priority of the throughput decoder (max-log): each wave publishes its
// progress (half SISOs since the launch) in a per-SIMD table indexed by HW_ID /
// XCC_ID and issues first while it is behind the other wave of its SIMD (the two
// otherwise issue oldest first, and with one tile each the younger runs its last
// ~3 ms alone at the one-wave rate: configs[1] 10.6 -> 9.8-9.9 ms per 102 400
// codewords, profiles/r03t/, r03z/).  Policies by tile progress or by pass, a finer
// comparison (4 units per SISO) and the same policy in the log-MAP decoder
// measured no better (profiles/r03x/, r03ab/, r03ac/).
__device__ __forceinline__ void set_prio(int v) {
    switch (v) {
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
    }
}
struct Prio {
    int *tab = nullptr;   // this SIMD's 16 progress slots (by wave id), or null
    int me = 0;           // this wave's slot
    int prog = 0;         // half SISOs completed before this SISO
};
__device__ __forceinline__ void mate_prio(const Prio &pr, int v) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) __hip_atomic_store(pr.tab + pr.me, v + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int x = lane < 16 ? __hip_atomic_load(pr.tab + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    if (lane == pr.me) x = 0;
    int mate = 0;
#pragma unroll
    for (int l = 0; l < 16; ++l) mate = max(mate, __builtin_amdgcn_readlane(x, l));
    set_prio(mate == 0 ? 2 : (v + 1 < mate ? 3 : (v + 1 > mate ? 1 : 2)));
}
constexpr int PRIO_UNITS = 2;   // progress units per SISO (forward half, backward half)
__device__ __forceinline__ void phase_prio(bool forward, const Prio &pr) {
    if (pr.tab) mate_prio(pr, pr.prog + (forward ? 0 : 1));
}

// The SISO with checkpoints every W steps (the row SISO, the fused demap-decode
// kernel and the log-MAP throughput decoder; max-log's throughput decoder runs
// siso8 below).
template <int ALGO, int W, bool RAG, class In, class Out>
__device__ void siso(const In &in, const Out &out, int N, float4 *ck, float4 *ring, unsigned cs, int lane,
                     double sf) {
    const int top = RAG ? ((N - 1) / W) * W : N - W;   // start of the (possibly short) top window
    constexpr int RSTEP = rstep_of(W);
    Raw raw[W];
    float a[NS], b[NS], an[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) a[s] = b[s] = 0.0f;
    if constexpr (ALGO != 0) {
        f1_pass<ALGO, W, RAG, false>(in, N, ck, cs, lane, a);   // a = alpha1[N] = alpha2[0]
        f1_pass<ALGO, W, RAG, true>(in, N, ck, cs, lane, a);    // alpha2, every checkpoint
        b1_pass<ALGO, RAG>(in, N, b);                           // b = beta1[0] = beta2[N]
#pragma unroll
        for (int j = 0; j < W; ++j) raw[j] = in.load(RAG ? min(top + j, N - 1) : top + j);
        load_vec<true>(an, ck, cs, (top / W) * 4, lane);
        for (int k0 = top; k0 >= 0; k0 -= W)
            back_window<ALGO, W, RAG>(in, out, k0, RAG ? min(W, N - k0) : W, raw, an, b, ck, cs, lane, N, sf);
        return;
    }
    // F1 (inputs software-pipelined one group of FG steps ahead)
    f1_pass<ALGO, W, RAG>(in, N, ck, cs, lane, a);
    // F2 until merged (a = alpha1[N] = alpha2[0]).  Per lane: once alpha2 ==
    // alpha1 at a checkpoint, every later checkpoint already holds alpha2, so
    // the lane stops loading and storing (masked lanes move no bytes); the
    // wave runs until every lane has merged.  (The unmasked form -- every lane
    // loads, merged lanes only skip stores -- measured slower for max-log: 66.7 vs
    // 64.6 ms per 262 144 codewords, round 2.)
#pragma unroll
    for (int j = 0; j < W; ++j) raw[j] = in.load(RAG ? min(j, N - 1) : j);
    bool merged = false;
    for (int k0 = 0; k0 < N; k0 += W) {
        if (!merged) merged = lane_equal<true>(a, ck, cs, (k0 / W) * 4, lane);
        if (__all(merged)) break;
        if (!merged) {
            float g[W][8];
#pragma unroll
            for (int j = 0; j < W; ++j) {
                double iA, iB;
                in.template gamma<ALGO>(raw[j], g[j], iA, iB);
            }
            if (k0 + W < N) {
#pragma unroll
                for (int j = 0; j < W; ++j) raw[j] = in.load(RAG ? min(k0 + W + j, N - 1) : k0 + W + j);
            }
            store_vec<true>(ck, cs, (k0 / W) * 4, lane, a);
#pragma unroll
            for (int j = 0; j < W; ++j)
                if (!RAG || k0 + j < N) alpha_step<ALGO>(a, g[j]);
        }
    }
    // B1 fused with the provisional extrinsic, then B2 until merged (b =
    // beta1[0] = beta2[N]); per lane as F2: below its merge point a lane's
    // provisional extrinsics are exact, it stops there.  One copy of the window
    // code serves both passes (the pass loop is not unrolled: the kernels'
    // instruction footprint, see siso8).
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int j = 0; j < W; ++j) raw[j] = in.load(RAG ? min(top + j, N - 1) : top + j);
        load_vec<true>(an, ck, cs, (top / W) * 4, lane);
        merged = false;
        for (int k0 = top; k0 >= 0; k0 -= W) {
            const int r = (top - k0) / W;                     // window index from the top
            const bool keep = r % RSTEP == 0 && r < RING * RSTEP;
            if (pass == 0) {
                if (keep) store_vec<false>(ring, cs, r / RSTEP * 4, lane, b);   // beta1 entering
            } else if (keep) {
                float rv[NS];
                load_vec<false>(rv, ring, cs, r / RSTEP * 4, lane);
                if (!merged) merged = vec_equal(b, rv);
                if (__all(merged)) break;
            }
            if (!merged)
                back_window<ALGO, W, RAG>(in, out, k0, RAG ? min(W, N - k0) : W, raw, an, b, ck, cs, lane, N, sf);
        }
    }
}


// ---- max-log SISO with alpha checkpoints every 8 steps ---------------------------
// Halves the checkpoint stream of siso<> (16 B per step -> 8 B written, and the
// same read back) at the cost of half an extra alpha step per position.  A
// backward window of 8 positions is processed as two halves of 4: the top half
// needs alpha[k0+4], i.e. 4 steps from the checkpoint over the BOTTOM half's
// inputs, which are needed again for the bottom half itself.  Those inputs are
// staged per lane in LDS (8 KiB per wave) by LDS-DMA (global_load_lds) issued
// one window ahead, so they cost no VGPRs.  Every value is computed by the same f32/f64 operations in
// the same order as siso<>, so the result is bit-identical.

// Positions kb+3 .. kb of a half window (kb+len-1 .. kb if ragged), alpha[kb]
// given, midpoint recompute as back_window.
template <int ALGO, bool RAG, class Out>
__device__ __forceinline__ void window_half(const Out &out, int kb, int len, const float (&a0)[NS],
                                            const float (&gw)[4][8], const double (&iAw)[4], const double (&iBw)[4],
                                            const float (&lcA)[4], const float (&lcB)[4], float (&b)[NS], double sf) {
    constexpr int H = 2;
    float am[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) am[s] = a0[s];
#pragma unroll
    for (int i = 0; i < H; ++i) alpha_step<ALGO>(am, gw[i]);
#pragma unroll
    for (int j = 3; j >= 0; --j) {
        if (RAG && j >= len) continue;       // wave-uniform
        __builtin_amdgcn_sched_barrier(0);
        const int from = j >= H ? H : 0;
        double leA = 0.0, leB = 0.0;
        if (out.need(kb + j)) {
            float aj[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                aj[s] = j >= H ? am[s] : a0[s];
                asm volatile("" : "+v"(aj[s]));
            }
#pragma unroll
            for (int i = from; i < j; ++i) alpha_step<ALGO>(aj, gw[i]);
            extrinsic<ALGO>(aj, gw[j], b, iAw[j], iBw[j], sf, leA, leB);
        }
        out.store(kb + j, leA, leB, lcA[j], lcB[j]);
        beta_step<ALGO>(b, gw[j]);
    }
}

// Window [k0, k0+len) of the backward sweep, len <= 8, in two halves of 4.
// On entry rt holds this window's top-half inputs, an its alpha checkpoint and
// st its bottom-half inputs (staged in LDS); on exit they hold the next (lower)
// window's (st / sn swap with the window parity).  Every load is issued a
// half window or more before its use and is unconditional (the last window
// re-reads its own rows), so the compiler's wait counts stay exact:
//   start:       top-half gammas from rt; DMA of the next bottom half into sn
//   wait:        st and an have landed (issued a window / half window ago)
//   top half:    alpha[k0+4] from the checkpoint over st; rt <- next top half
//   bottom half: gammas from st; an <- next checkpoint
// The window's checkpoint is DMA'd into the wave's LDS slot (st.ck) at the
// previous window's bottom half, after that window's last read of the slot,
// and read from it twice (alpha[k0+4] and the bottom half), so it holds no
// registers across the top half.
__device__ __forceinline__ void ck_stage(const float4 *ck, unsigned cs, unsigned base, int lane, lds_f4 *slot) {
#pragma unroll
    for (int q = 0; q < 4; ++q) glds16s(ck, ((base + q) * cs + lane) * 16u, slot + q * WAVE);
}
__device__ __forceinline__ void ck_read(const lds_f4 *slot, int lane, float (&x)[NS]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = ld4(slot + q * WAVE + lane);
        x[vec_elem<true>(q, 0)] = v.x;
        x[vec_elem<true>(q, 1)] = v.y;
        x[vec_elem<true>(q, 2)] = v.z;
        x[vec_elem<true>(q, 3)] = v.w;
    }
}
template <int ALGO, bool RAG, class In, class Out>
__device__ __forceinline__ void back_window8(const In &in, const Out &out, int k0, int len, Raw (&rt)[4],
                                             const LdsStage &st, const LdsStage &sn,
                                             float (&b)[NS], const float4 *ck, unsigned cs, int lane, int N,
                                             double sf) {
    const int lenT = RAG ? (len > 4 ? len - 4 : 0) : 4;
    const int lenB = RAG ? (len < 4 ? len : 4) : 4;
    const int kn = k0 >= 8 ? k0 - 8 : 0;   // the next window
    float gw[4][8], lcA[4], lcB[4];
    double iAw[4], iBw[4];
    if (!RAG || lenT > 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            in.template gamma<ALGO>(rt[j], gw[j], iAw[j], iBw[j]);
            lcA[j] = rt[j].v.x;
            lcB[j] = rt[j].v.y;
        }
    }
    // (The last window re-reads its own rows here: skipping that saves 4 KB per
    // codeword, L2-resident anyway, and measured neutral, profiles/r06/b/.)
#pragma unroll
    for (int j = 0; j < 4; ++j) in.stage(RAG ? min(kn + j, N - 1) : kn + j, sn, j);
    in.wait_staged();   // + 4 for the checkpoint DMA, issued before the stage just above
    // (Keeping alpha[k0+2], passed on the way to alpha[k0+4], for the bottom half's
    // midpoint measured slower: profiles/r03w/, 250.9 vs 244.2 ms per 1 M codewords,
    // configs[1] 14.0 vs 10.4 ms -- the 16 registers it holds across the top half
    // cost more than the two alpha steps it saves.)
    if (!RAG || lenT > 0) {
        float a4[NS];    // alpha[k0+4]: 4 steps from the checkpoint over the staged bottom half
        ck_read(st.ck, lane, a4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float g[8];
            double x, y;
            in.template gamma<ALGO>(in.staged(st, i), g, x, y);
            alpha_step<ALGO>(a4, g);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) rt[j] = in.load(RAG ? min(kn + 4 + j, N - 1) : kn + 4 + j);
        window_half<ALGO, RAG>(out, k0 + 4, lenT, a4, gw, iAw, iBw, lcA, lcB, b, sf);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) rt[j] = in.load(RAG ? min(kn + 4 + j, N - 1) : kn + 4 + j);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const Raw r = in.staged(st, j);
        in.template gamma<ALGO>(r, gw[j], iAw[j], iBw[j]);
        lcA[j] = r.v.x;
        lcB[j] = r.v.y;
    }
    float a0[NS];
    ck_read(st.ck, lane, a0);
    // The slot's last read must have returned before the DMA that overwrites it is
    // issued: the ISA does not order an outstanding ds_read against a later LDS-DMA
    // write, and the compiler's wait-count pass cannot see the asm DMA.  a0 is
    // needed at once by the bottom half, so the wait costs nothing.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ck_stage(ck, cs, (kn / 8) * 4, lane, st.ck);
    window_half<ALGO, RAG>(out, k0, lenB, a0, gw, iAw, iBw, lcA, lcB, b, sf);
}

// beta1 kept at every 2nd window start: the same 16-step grid over the top 256
// steps as siso<>.  (An 8-step grid over the top 128 steps -- B2 stops up to 8 steps
// earlier for the same ring writes -- measured neutral at N = 212 and slower at
// 752, where lanes merging below the top 128 steps run B2 to the end.)
constexpr int RSTEP8 = 2;

// TDEC_PASS_TIMING (measurement build): per-pass shader-clock cycles summed
// over all waves (s_memtime, one vector atomic from lane 0 per pass), printed
// by tdec_destroy: [0] F1, [1] F2, [2] B1, [3] B2, [4] epilogue.
#ifndef TDEC_PASS_TIMING
#define TDEC_PASS_TIMING 0
#endif
// The same build also histograms where the merge passes end:
// g_merge_hist[0] F2 per lane, [1] F2 per wave (its deepest lane), in units of
// 8-step checkpoints from k = 0; [2] B2 per lane, [3] B2 per wave, in 8-step
// windows from the top.  Bucket MH_END: never merged (ran to the end).
constexpr int MH_END = 127;
#if TDEC_PASS_TIMING
__device__ unsigned long long g_pass_cycles[8];
__device__ unsigned long long g_merge_hist[4][MH_END + 1];
__device__ __forceinline__ void pass_mark(unsigned long long &t, int slot) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & (WAVE - 1)) == 0) atomicAdd(&g_pass_cycles[slot], now - t);
    t = now;
}
__device__ __forceinline__ void merge_mark(int which, int lane_at, int wave_at) {
    atomicAdd(&g_merge_hist[which][min(lane_at, MH_END)], 1ull);
    if ((threadIdx.x & (WAVE - 1)) == 0) atomicAdd(&g_merge_hist[which + 1][min(wave_at, MH_END)], 1ull);
}
#else
__device__ __forceinline__ void pass_mark(unsigned long long &, int) {}
__device__ __forceinline__ void merge_mark(int, int, int) {}
#endif

template <int ALGO, bool RAG, class In, class Out>
__device__ void siso8(const In &in, const Out &out, int N, float4 *ck, float4 *ring, unsigned cs, int lane, double sf,
                      const LdsStage &lb, const LdsStage &lb1, const Prio &pr = Prio{}) {
    unsigned long long tpass = TDEC_PASS_TIMING ? __builtin_amdgcn_s_memtime() : 0;
    phase_prio(true, pr);
    constexpr int G = 4, WS = 8, CK = 8;   // group, window step, checkpoint interval
    const int top = RAG ? ((N - 1) / WS) * WS : N - WS;
    Raw raw[G];
    float a[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) a[s] = 0.0f;
    // F1: inputs pipelined one group of FG steps ahead, checkpoint every 8
    f1_pass<ALGO, WS, RAG, true>(in, N, ck, cs, lane, a);
    pass_mark(tpass, 0);
    // F2 until merged with F1 at a checkpoint.  (Measured alternative, round 2:
    // the next checkpoint prefetched one interval ahead with unmasked input
    // loads cut F2's share of wave time from 7.4 to 5.6 % but the extra bytes
    // made the decode 1.1 % slower.)
#pragma unroll
    for (int j = 0; j < G; ++j) raw[j] = in.load(RAG ? min(j, N - 1) : j);
    bool merged = false;   // per lane, as siso<>
    int mlane = MH_END, mwave = MH_END;   // TDEC_PASS_TIMING: merge checkpoints
    for (int k0 = 0; k0 < N; k0 += G) {
        const bool at_ck = (k0 & (CK - 1)) == 0;
        if (at_ck) {
            if (!merged) {
                merged = lane_equal<true>(a, ck, cs, (k0 / CK) * 4, lane);
                if (TDEC_PASS_TIMING && merged) mlane = k0 / 8;
            }
            if (__all(merged)) {
                mwave = k0 / 8;
                break;
            }
        }
        if (!merged) {
            float g[G][8];
#pragma unroll
            for (int j = 0; j < G; ++j) {
                double iA, iB;
                in.template gamma<ALGO>(raw[j], g[j], iA, iB);
            }
            if (k0 + G < N) {
#pragma unroll
                for (int j = 0; j < G; ++j) raw[j] = in.load(RAG ? min(k0 + G + j, N - 1) : k0 + G + j);
            }
            if (at_ck) store_vec<true>(ck, cs, (k0 / CK) * 4, lane, a);
#pragma unroll
            for (int j = 0; j < G; ++j)
                if (!RAG || k0 + j < N) alpha_step<ALGO>(a, g[j]);
        }
    }
    pass_mark(tpass, 1);
    merge_mark(0, mlane, mwave);
    phase_prio(false, pr);
    // B1 fused with the provisional extrinsic, then B2 until merged (as siso<>)
    float b[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) b[s] = 0.0f;
    // B1 and B2 share one copy of the window code (the pass loop is not
    // unrolled), halving the backward sweep's instruction footprint: the kernel
    // shrinks from 15.2 k to 9.6 k instructions and decodes 1.5 % faster (62.6 ->
    // 61.7 ms per 262 144 codewords, same bits): the waves of a CU run different
    // passes at once and share its instruction cache.
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
        // The lane index goes through an empty asm here, so the per-lane addresses
        // of this prologue are formed from it again (a shift and an add each)
        // instead of hoisted out of the tile's loops and spilled: the spilled ones
        // came back through scratch loads, each followed by a full vmcnt(0) wait
        // ahead of the DMA that needed it.
        In inp = in;
        int lanep = lane;
        asm volatile("" : "+v"(inp.lane), "+v"(lanep));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            raw[j] = inp.load(RAG ? min(top + 4 + j, N - 1) : top + 4 + j);
            inp.stage(RAG ? min(top + j, N - 1) : top + j, lb, j);
        }
        ck_stage(ck, cs, (top / CK) * 4, lanep, lb.ck);
        merged = false;
        mlane = mwave = MH_END;
        for (int k0 = top; k0 >= 0; k0 -= WS) {
            const int r = (top - k0) / WS;
            const bool keep = r % RSTEP8 == 0 && r < RING * RSTEP8;
            if (pass == 0 && keep) store_vec<false>(ring, cs, r / RSTEP8 * 4, lane, b);   // beta1 entering
            if (pass == 1 && keep) {
                if (!merged) {
                    merged = lane_equal<false>(b, ring, cs, r / RSTEP8 * 4, lane);
                    if (TDEC_PASS_TIMING && merged) mlane = r;
                }
                if (__all(merged)) {
                    mwave = r;
                    break;
                }
            }
            if (!merged) {
                const bool odd = r & 1;
                back_window8<ALGO, RAG>(in, out, k0, RAG ? min(WS, N - k0) : WS, raw, odd ? lb1 : lb,
                                        odd ? lb : lb1, b, ck, cs, lane, N, sf);
            }
        }
        pass_mark(tpass, 2 + pass);
    }
    merge_mark(2, mlane, mwave);
}

// ---- kernels --------------------------------------------------------------------
constexpr int BLOCK = 256;               // 4 waves; each wave owns one 64-codeword tile at a time
constexpr int WAVES_PER_BLOCK = BLOCK / WAVE;
// Waves per block of the tile decoders (k_turbo_decode, k_turbo_decode_logmap).
// The waves of a block are independent (no barrier), so the block size only
// decides how the dispatcher can spread waves over CUs: with fewer tiles than
// wave slots (one round, e.g. configs[1]: 1 600 tiles for 2 048 slots) four-wave
// blocks leave some CUs with 8 waves and others with 4, and the launch lasts as
// long as the fullest CU (a CU's memory pipeline, not its SIMDs, is what a tile
// waits on: profiles/r03p/c1_batch_sweep.txt; one- and four-wave blocks measured equal).
constexpr int DEC_WAVES = 4;
constexpr int DEC_BLOCK = DEC_WAVES * WAVE;
constexpr int WIN = 4;                   // alpha checkpoint interval of the row SISO (k_siso_batch)
// max-log checkpoint interval of k_turbo_decode: 8 (siso8: LDS-DMA staged half
// windows, bit-identical to siso<> at 4).  8 moves 13 % fewer bytes per codeword;
// it was slower (round 1: 73.7 vs 69.8 ms per 262 144 codewords) until its loads
// were issued a half window or more ahead with exact wait counts (inline-asm LDS
// DMA, checkpoint slot in LDS, 32-bit LDS pointers): round 2, 62.4 vs 65.0 ms
// (tools/ab.py, same bits).  16 measured slower.
constexpr int WIN_ML = 8;
constexpr int WIN_LM = 2;                // log-MAP turbo decoder's checkpoint interval
__host__ __device__ constexpr int win_of(int algo) { return algo ? WIN_LM : WIN_ML; }
constexpr int LDS_STAGE1 = DEC_WAVES * 4 * WAVE;   // float4 / double2 entries of one staging buffer of a block
constexpr int LDS_STAGE = LDS_STAGE1 * 2;   // double-buffered (siso8)
// siso8's LDS per block: lv = 2 staging buffers + the checkpoint slots (float4),
// ll = 2 staging buffers (double2): 20 KiB per wave, eight waves per CU.  The epilogue's
// bit-packing words then live in the wave's own first staging slice (idle
// between tiles) instead of a separate array that would not fit.
constexpr int LDS_LV = LDS_STAGE + DEC_WAVES * 4 * WAVE;
constexpr int EPI_STRIDE_ML = 4 * WAVE * 4;   // uint32 words between waves' epi areas

// The SISO of the tile decoder: siso8 (LDS-staged, checkpoints every 8) for
// max-log when the kernel provides the staging LDS (STAGED), else siso<> with
// checkpoints every 4 (max-log, the fused demap-decode kernel) or WIN_LM.
__host__ __device__ constexpr int win_unstaged(int algo) { return algo ? WIN_LM : 4; }
// A handle's checkpoint rows are sized for the densest interval among the kernels
// that can run for its algorithm: the row SISO (WIN), the tile decoder
// (win_of) and the fused demap-decode kernel (win_unstaged).
__host__ __device__ constexpr int cmin(int a, int b) { return a < b ? a : b; }
__host__ __device__ constexpr int ck_win_of(int algo) { return cmin(WIN, cmin(win_of(algo), win_unstaged(algo))); }
template <int ALGO, bool RAG, bool STAGED, class In, class Out>
__device__ __forceinline__ void run_siso(const In &in, const Out &out, int N, float4 *ck, float4 *ring, unsigned cs,
                                         int lane, double sf, float4 *lv, double2 *ll, const Prio &pr = Prio{}) {
    if constexpr (ALGO == 0 && STAGED) {
        const int w = threadIdx.x >> 6;
        lds_f4 *v = (lds_f4 *)lv;
        lds_d2 *l = (lds_d2 *)ll;
        lds_f4 *slot = v + LDS_STAGE + w * 4 * WAVE;
        siso8<ALGO, RAG>(in, out, N, ck, ring, cs, lane, sf, LdsStage{v + w * 4 * WAVE, l + w * 4 * WAVE, lane, slot},
                         LdsStage{v + LDS_STAGE1 + w * 4 * WAVE, l + LDS_STAGE1 + w * 4 * WAVE, lane, slot}, pr);
    } else {
        siso<ALGO, (ALGO ? WIN_LM : 4), RAG>(in, out, N, ck, ring, cs, lane, sf);
    }
}

// Plane layout of one 64-codeword tile ([N][64] each, codeword fastest):
//   X[k] = {A[k], B[k], W1[k], Y1[k]}  float4   decoder 1, natural order
//   Z[k] = {W2[k], Y2[k]}              float2   decoder 2's parities
// 24 B per trellis step and codeword: exactly the de-punctured LLRs.
__host__ __device__ constexpr long tile_floats(int N) { return (long)N * WAVE * 6; }

struct DecodeArgs {
    int B, N, iters, n_tiles, n_waves;
    const float *planes;     // [n_tiles] x (X, Z)
    double2 *ws;             // [3][N][n_waves][64]: P1, Le2, Le1 (last iteration)
    float4 *ck;              // [ck_rows + RING][4][n_waves][64]: alpha checkpoints, beta1 ring
    int32_t *bits;           // [B][2N]
    double *lfinal;          // [B][2N] or null
    const int *p1_used;      // [N]: 1 where k is in the image of perm (P1 rows decoder 2 reads)
    // workspace row stride in lanes (= n_waves * 64, set by the host): opaque to the
    // compiler, which otherwise proves it a multiple of 64 and forms every lane
    // offset with v_lshlrev + v_or instead of one v_add_lshl_u32 (+1.5 % decode time)
    int row_lanes;
    double2 *aux;            // [64] zeros (the first iteration's a-priori), then one sink row per wave
    int *tile_ctr;           // null: static tile striding; else a zeroed counter (dynamic tile queue)
    int ck_rows;             // checkpoint rows before the beta1 ring: ceil(N / ck_win_of(algo))
    int *simd_prog = nullptr;   // max-log issue priority: [8192 SIMDs][16 wave slots] progress, zeroed per launch
    // The launch's tail: once the last tile has been handed out (the dynamic tile
    // counter is exhausted, or, with static striding, the wave of the highest tile
    // starts it) that wave raises *tail_flag to tail_seq (atomicMax; seq grows per
    // launch), which k_tail_gate waits for (tdec_tail_gate: the next batch's demap
    // is released into the slots the retiring waves free, not before the grid is
    // placed).  Approximate by nature: with static striding other waves may still
    // be starting their last tiles of the same round, and a launch captured in a
    // graph keeps its tail_seq, so on replay the gate finds the flag already raised.
    unsigned *tail_flag = nullptr;
    unsigned tail_seq = 0;
};

// DVBRCS2_Turbo.decode (:464-537) for 64 codewords per wave, persistent over tiles.
// Where a tile's planes come from.  PlanesIn: the caller's plane buffer
// (tdec_decode_planes_dev); fill / publish are no-ops.  The fused demap
// (DemapPro, below) fills a wave's next tile piece by piece between the SISOs of
// the current one, into the other of its two plane buffers.
struct PlanesIn {
    const float *planes;
    __device__ __forceinline__ const float *tile_planes(int tile, int /*wave*/, int N, int /*buf*/) const {
        return planes + (long)tile * tile_floats(N);
    }
    __device__ __forceinline__ void fill(int, int, int, int, int, int) const {}
    __device__ __forceinline__ void publish() const {}
};

// TDEC_WAVE_TIMING (measurement build): per persistent wave of the last decode
// launch, {first, last} s_memrealtime (100 MHz, chip-wide) and {first, last}
// s_memtime (shader clock), the tiles it took and its HW_ID / XCC_ID, printed by
// tdec_destroy (TDEC_WAVE_DUMP: per wave, tools/wave_dump.py): how much of the
// launch the waves spend idle in the tail, and the clock each wave ran at
// (shader ticks / real time).
#ifndef TDEC_WAVE_TIMING
#define TDEC_WAVE_TIMING 0
#endif
#if TDEC_WAVE_TIMING
constexpr int WT_MAX = 16384;
__device__ unsigned long long g_wave_t[WT_MAX][4];   // realtime start, end; memtime start, end
__device__ int g_wave_tiles[WT_MAX];
__device__ unsigned g_wave_hw[WT_MAX][2];   // HW_ID (wave, SIMD, CU, SH, SE fields) and XCC_ID of each wave
#endif

// One tile = 64 codewords, one per lane.  (Sub-tile units -- every resident wave
// one unit of ceil(B / waves) < 64 codewords when a batch has more tiles than SIMDs
// but fewer than resident waves, so every SIMD holds two equally loaded waves --
// measured slower at configs[1]: 10.74 vs 9.65 ms per 102 400 codewords, the clock
// 1.68 vs 1.83 GHz: the extra waves' instruction streams cost more power than the
// balance saved, profiles/r06a/, DESIGN.md appendix.)
template <int ALGO, bool RAG, bool STAGED = false, class Pro = PlanesIn>
__device__ __forceinline__ void turbo_decode_tiles(const DecodeArgs &p, const int *__restrict__ perm,
                                                   const int *__restrict__ inv, const int *__restrict__ used,
                                                   float4 *lv, double2 *ll,
                                                   uint32_t *epi, const Pro &pro = Pro{}, int epi_stride = 2 * WAVE) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (wave >= p.n_waves) return;
    const int N = p.N;
    const long NW = (long)N * WAVE;
    // workspace rows interleave the waves: [plane][k][wave][64] and [slot][wave][64]
    const unsigned rs = (unsigned)p.row_lanes;
    double2 *P1 = p.ws + (long)wave * WAVE * WS_G, *Le2 = P1 + (long)rows_of(N) * rs, *Le1 = Le2 + (long)rows_of(N) * rs;
    const int nw = p.ck_rows;
    float4 *ck = p.ck + (long)wave * WAVE * WS_G;
    float4 *ring = ck + (long)nw * 4 * rs;
    double2 *sink = p.aux + WAVE + (long)wave * WAVE;
    int buf = 0;
#if TDEC_WAVE_TIMING
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime(), wc0 = __builtin_amdgcn_s_memtime();
    int wtiles = 0;
#endif
    pro.fill(wave, wave, N, 0, 0, 1);   // the first tile whole; later ones during the previous tile
    pro.publish();
    Prio pr;
    if (p.simd_prog) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
        const unsigned key = ((xcc & 7u) << 10) | (((hw >> 13) & 7u) << 7) | (((hw >> 12) & 1u) << 6) |
                             (((hw >> 8) & 15u) << 2) | ((hw >> 4) & 3u);
        pr.tab = p.simd_prog + key * 16;
        pr.me = (int)(hw & 15u);
    }
    // Every wave starts with tile `wave`; with a tile counter the next tile is
    // taken from a queue (one atomic per tile from lane 0, issued at the tile's
    // start, consumed at its end), so waves whose codewords take longer (longer
    // merge passes) take fewer tiles and all waves finish close together.
    // (A queue of (tile, iteration) items instead of whole tiles, per-XCD rings with
    // Le2 handed between waves, measured no faster: DESIGN.md, appendix.)
    // One trip of this loop per (tile, iteration); the SISO call sites exist once
    // (the kernel's instruction footprint is shared by the CU's waves).
    int tile = wave, it = 0, nxt = 0;
    bool has_next = false;
    for (;;) {
        if (tile >= p.n_tiles) break;
        if (it == 0) {
            nxt = tile + p.n_waves;
            if (p.tile_ctr) {
                int q = 0;
                if (lane == 0) q = atomicAdd(p.tile_ctr, 1);
                nxt = p.n_waves + __builtin_amdgcn_readfirstlane(q);
            }
            has_next = nxt < p.n_tiles;
            if (p.tail_flag && lane == 0 && (p.tile_ctr ? !has_next : tile == p.n_tiles - 1))
                atomicMax(p.tail_flag, p.tail_seq);
        }
        const float *base = pro.tile_planes(tile, wave, N, buf);
        const float4 *X = reinterpret_cast<const float4 *>(base);
        const float2 *Z = reinterpret_cast<const float2 *>(base + NW * 4);
        {
            const double sf = it < p.iters - 1 ? 0.7 : 1.0;     // :496
            const bool last = it == p.iters - 1;
            run_siso<ALGO, RAG, STAGED>(TileIn{X, it ? Le2 : p.aux, inv, lane, it ? rs : 0u},
                                        TileOutPre{P1, last ? Le1 : nullptr, lane, rs, used, sink}, N, ck, ring, rs,
                                        lane, sf, lv, ll, pr);
            pr.prog += PRIO_UNITS;
            if (has_next) pro.fill(nxt, wave, N, buf ^ 1, 2 * it, 2 * p.iters);
            run_siso<ALGO, RAG, STAGED>(TileInPre{Z, P1, perm, lane, rs}, TileOut{Le2, lane, rs}, N, ck, ring, rs, lane,
                                        sf, lv, ll, pr);
            pr.prog += PRIO_UNITS;
            if (has_next) pro.fill(nxt, wave, N, buf ^ 1, 2 * it + 1, 2 * p.iters);
        }
        if (it < p.iters - 1) {
            ++it;
            continue;
        }
        unsigned long long tepi = TDEC_PASS_TIMING ? __builtin_amdgcn_s_memtime() : 0;
        // hard decision (:526-537): L = (Lc + La) + Le1, La = Le2[inv_perm].
        // Bits of 32 couples per lane are packed into two LDS words, then the wave
        // writes the 64 rows chunk by chunk in row order (16-B int4 stores, each
        // wave store one contiguous 1 KiB run) instead of one 8-B store per lane
        // per couple 6 KB apart.
        const long cw = (long)tile * WAVE + lane;
        const bool lane_on = cw < p.B;
        uint32_t *hb = epi + (threadIdx.x >> 6) * epi_stride;
        const long nb = 2L * N;
        for (int kc = 0; kc < N; kc += 32) {
            uint32_t w0 = 0, w1 = 0;
            double *lo = (p.lfinal && lane_on) ? p.lfinal + cw * nb : nullptr;
            const int kn = min(32, N - kc);
            // groups of 8 steps whose 24 loads are issued together (one exposed
            // memory latency per group, not per step; 3.2 % of the decode before)
            for (int kg = 0; kg < kn; kg += 8) {
                float2 xa[8];
                double2 la[8], le[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int k = min(kc + kg + u, N - 1);   // past the chunk: a valid row, unused
                    const float4 x = at(X, k * WAVE + lane);
                    xa[u] = make_float2(x.x, x.y);
                    la[u] = at(Le2, wsrow(inv[k], rs) + lane);
                    le[u] = at(Le1, wsrow(k, rs) + lane);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int kk = kg + u, k = kc + kk;
                    if (kk >= kn) break;   // wave-uniform
                    const double fa = ((double)xa[u].x + la[u].x) + le[u].x;
                    const double fb = ((double)xa[u].y + la[u].y) + le[u].y;
                    const uint32_t two = (fa < 0.0 ? 1u : 0u) | (fb < 0.0 ? 2u : 0u);
                    if (kk < 16) w0 |= two << (2 * kk);
                    else w1 |= two << (2 * (kk - 16));
                    if (lo) *reinterpret_cast<double2 *>(lo + 2 * k) = make_double2(fa, fb);
                }
            }
            hb[lane] = w0;
            hb[WAVE + lane] = w1;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // 64 rows x 2*kn int32 of this chunk: item t = (row, 4-bit piece)
            const int per = (2 * kn + 3) / 4;
            for (int t = lane; t < WAVE * per; t += WAVE) {
                const int l = t / per, pc = t - l * per;
                const long row = (long)tile * WAVE + l;
                if (row >= p.B) continue;
                const uint32_t w = hb[(pc >> 3) * WAVE + l] >> (4 * (pc & 7));
                const int j = 4 * pc;                          // first int32 of the piece within the chunk
                int32_t *dst = p.bits + row * nb + 2L * kc + j;
                if (j + 4 <= 2 * kn && (nb & 3) == 0)
                    *reinterpret_cast<int4 *>(dst) = make_int4(w & 1, (w >> 1) & 1, (w >> 2) & 1, (w >> 3) & 1);
                else
                    for (int e = 0; e < 4 && j + e < 2 * kn; ++e) dst[e] = (w >> e) & 1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        pass_mark(tepi, 4);
        if (has_next) pro.publish();
        buf ^= 1;
        tile = nxt;
        it = 0;
#if TDEC_WAVE_TIMING
        ++wtiles;
#endif
    }
    if (pr.tab && lane == 0) __hip_atomic_store(pr.tab + pr.me, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if TDEC_WAVE_TIMING
    if (lane == 0 && wave < WT_MAX) {
        g_wave_t[wave][0] = wt0;
        g_wave_t[wave][1] = __builtin_amdgcn_s_memrealtime();
        g_wave_t[wave][2] = wc0;
        g_wave_t[wave][3] = __builtin_amdgcn_s_memtime();
        g_wave_tiles[wave] = wtiles;
        g_wave_hw[wave][0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        g_wave_hw[wave][1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
    }
#endif
}

// Both held to 256 registers (2 waves per SIMD).  max-log: the few tile-level
// values that do not fit go to scratch, outside the trellis loops.  log-MAP
// spills more (its max* needs the registers), but a second wave per SIMD still
// beats the one-wave VALU issue limit by a third.
// (Three waves per SIMD for log-MAP -- 168 VGPRs, loops without spills -- measured
// slower: 141.9 vs 122.3 ms per 262 144 codewords, profiles/r05/lm3_ab/.)
constexpr int DEC_WPE = 2;
template <bool RAG>
__global__ __launch_bounds__(DEC_BLOCK) __attribute__((amdgpu_waves_per_eu(DEC_WPE))) void k_turbo_decode(
    DecodeArgs p, const int *__restrict__ perm, const int *__restrict__ inv, const int *__restrict__ used) {
    __shared__ float4 lv[LDS_LV];
    __shared__ double2 ll[LDS_STAGE];
    turbo_decode_tiles<0, RAG, true>(p, perm, inv, used, lv, ll, reinterpret_cast<uint32_t *>(lv), PlanesIn{p.planes},
                                     EPI_STRIDE_ML);
}
template <bool RAG>
__global__ __launch_bounds__(DEC_BLOCK) __attribute__((amdgpu_waves_per_eu(DEC_WPE))) void k_turbo_decode_logmap(
    DecodeArgs p, const int *__restrict__ perm, const int *__restrict__ inv, const int *__restrict__ used) {
    __shared__ uint32_t epi[DEC_WAVES * 2 * WAVE];
    turbo_decode_tiles<1, RAG>(p, perm, inv, used, nullptr, nullptr, epi, PlanesIn{p.planes});
}

// One SISO over B codewords given as [B][N] rows (the bcjr_max_log_map boundary).
// Channel LLRs as float32 (Lc*) or, for the F64 kernels, float64 (Lc64*).
struct SisoArgs {
    int B, N, n_waves;
    const float *LcA, *LcB, *LcW, *LcY;
    const double *LaA, *LaB;
    double sf;
    double *LeA, *LeB;
    float4 *ck;
    long ck_stride;
    const double *Lc64A, *Lc64B, *Lc64W, *Lc64Y;
};

template <int ALGO, bool RAG, bool F64> __device__ __forceinline__ void siso_rows(const SisoArgs &p) {
    const int lane = threadIdx.x & (WAVE - 1);
    const int wave = __builtin_amdgcn_readfirstlane(blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6));
    if (wave >= p.n_waves) return;
    const long cw = (long)wave * WAVE + lane;
    const long row = (cw < p.B ? cw : p.B - 1) * p.N;     // idle lanes recompute the last row, store nothing
    const int nw = (p.N + WIN - 1) / WIN;
    float4 *ck = p.ck + (long)wave * p.ck_stride;
    const RowOut out{p.LeA + row, p.LeB + row, cw < p.B};
    if constexpr (F64) {
        RowIn64 in{p.Lc64A + row, p.Lc64B + row, p.Lc64W + row, p.Lc64Y + row, p.LaA + row, p.LaB + row};
        siso<ALGO, WIN, RAG>(in, out, p.N, ck, ck + (long)nw * 4 * WAVE, WAVE, lane, p.sf);
    } else {
        RowIn in{p.LcA + row, p.LcB + row, p.LcW + row, p.LcY + row, p.LaA + row, p.LaB + row};
        siso<ALGO, WIN, RAG>(in, out, p.N, ck, ck + (long)nw * 4 * WAVE, WAVE, lane, p.sf);
    }
}
template <bool RAG, bool F64 = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(2))) void k_siso_batch(SisoArgs p) {
    siso_rows<0, RAG, F64>(p);
}
template <bool RAG, bool F64 = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(DEC_WPE))) void k_siso_batch_logmap(
    SisoArgs p) {
    siso_rows<1, RAG, F64>(p);
}

// De-puncture (:468-487): llr rows -> tile planes X {A, B, W1, Y1} and Z {W2, Y2}.
// src[c*N + k] = LLR index or -1 for the components c = X.xyzw, (unused, unused), Z.xy.
// tdec_tail_gate: one wave that returns once *flag >= seq (a decoder launch has
// handed out its last tiles), polled with agent-scope loads (the flag is raised by
// atomics from any XCD) every ~4 us; after ~2 s it returns anyway (a late gate
// only costs overlap, never correctness).
__global__ __launch_bounds__(WAVE) void k_tail_gate(const unsigned *flag, unsigned seq) {
    for (unsigned i = 0; i < (1u << 19); ++i) {
        if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= seq) return;
        __builtin_amdgcn_s_sleep(127);
    }
}

__global__ __launch_bounds__(BLOCK) void k_depuncture(int B, int N, const float *llr, long stride,
                                                     const int *__restrict__ src, float *planes, long total) {
    const long t = (long)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= total) return;                 // total = tiles * N * 64
    const int lane = (int)(t & (WAVE - 1));
    const long q = t >> 6;                  // (tile, k): wave-uniform, so src[] is read by scalar loads
    const int k = __builtin_amdgcn_readfirstlane((int)(q % N));
    const long tile = __builtin_amdgcn_readfirstlane((int)(q / N));
    const long cw = tile * WAVE + lane;
    float v[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    if (cw < B) {
        const float *row = llr + cw * stride;
        const int comp[6] = {0, 1, 2, 3, 6, 7};
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            const int j = src[(long)comp[c] * N + k];
            if (j >= 0) v[c] = row[j];
        }
    }
    float *base = planes + tile * tile_floats(N);
    reinterpret_cast<float4 *>(base)[(long)k * WAVE + lane] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float2 *>(base + (long)N * WAVE * 4)[(long)k * WAVE + lane] = make_float2(v[4], v[5]);
}

// ---- soft demapper (compute_llr, test_sdr_with_coding.py:200-225) -----------------
// numpy's complex |z|: npmath.hip
using npm::cabs_np;

struct DemapCfg {
    int M, div_f32, sign;
    double nv;                 // max(noise_var, 0.005) already applied (:202)
    int sep;                   // 1: separable square QAM grid (per-axis levels follow the points);
                               // 2: and each axis a Gray-labelled uniform PAM (position-ordered levels follow)
    int nv_fast;               // nv in [2^-8, 2^16]: the unscaled f32 / f64 division (dm_fast)
};
__host__ __device__ inline int dm_nv_fast(double nv) { return nv >= 0x1p-8 && nv <= 0x1p16; }
// LDS table: 2*M point coordinates (+ 2 * 2^(bps/2) axis levels in label order; for a
// uniform grid labelled through gray[], sep == 2, + the levels in position order, 4
// parameters and the 2 * K * 2^K neighbour positions of sym_llrs_gray)
constexpr int DM_TAB = 768;

// The unscaled sequences (dm_fast): the compiler's own f64 division and square root
// sequences without their range scaling, where the scaling is provably the
// identity -- the same instructions on the same values, so the same bits:
//   a / b: v_div_scale (identity) -> r = v_rcp_f64(b), two Newton steps
//   r += r * (1 - b r), q = a r, rem = a - b q, q += rem r (v_div_fmas without its
//   2^64 scale), v_div_fixup (identity for finite nonzero operands and a normal
//   quotient); v_div_scale scales only for a denormal or huge denominator, a
//   numerator below 2^-969, a quotient below 2^-1022 or an exponent difference
//   >= 768;
//   sqrt(x), x in [1, 2]: y = v_rsq_f64(x), g = x y, h = y / 2, one Goldschmidt
//   step and two corrections (the 2^256 pre-scale applies below 2^-767 and the
//   zero / inf class select never fires).
// Outside those ranges the compiler's sequences run (a branch no lane takes on
// ordinary symbols).  tdec_selftest 4 compares both against the compiler's
// sequences on random operands over the ranges the demapper meets.
// BPSK .. 16QAM (measured faster, profiles/r05/demap_ab/); the 64 / 256QAM kernels
// keep the compiler's sequences (their registers grow past an occupancy step)
__host__ __device__ constexpr bool dm_fast(int bps) { return bps <= 4; }
__device__ __forceinline__ double rcp_nr64(double b) {   // v_div_scale-free reciprocal of the division sequence
    double r = __builtin_amdgcn_rcp(b);
    r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
    return __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
}
__device__ __forceinline__ double div_nr64(double a, double b, double r) {   // a / b given r = rcp_nr64(b)
    const double q = a * r;
    return __builtin_fma(__builtin_fma(-b, q, a), r, q);
}
// The f32 division the same way (v_div_scale_f32 scales for a denormal or huge
// denominator, a numerator below 2^-104, a denormal quotient or an exponent
// difference >= 96): r = v_rcp_f32(b), one Newton step, q = a r, two corrections
// (the second is v_div_fmas_f32 without its scale).
__device__ __forceinline__ float rcp_nr32(float b) {
    const float r = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
}
__device__ __forceinline__ float div_nr32(float a, float b, float r) {   // a / b given r = rcp_nr32(b)
    float q = a * r;
    q = __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
    return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
}
__device__ __forceinline__ double sqrt_1_2_64(double x) {   // sqrt(x) for x in [1, 2]
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
// One LLR from the two per-half minima (:219-225): NaN propagates, then the
// division by the noise variance, the +-30 clip and the caller's sign.
// PRE: the caller has checked nv_fast and that |diff| lies in the unscaled range
// (sym_llrs_pairs16), so the unscaled division runs without a per-LLR test.
// F32OUT (PRE only): the caller keeps the LLR as f32 (the plane kernels), so the
// f64 quotient is rounded first and clipped / negated in f32: the same value, since
// +-30 are f32 values, rounding is monotone and the quotient is finite here.
template <typename T, bool FAST = false, bool PRE = false, bool F32OUT = false>
__device__ __forceinline__ double llr_from_diff(T diff, const DemapCfg &c) {
    if constexpr (PRE) {
        if (sizeof(T) == 4 && c.div_f32) {
            const float fn = (float)c.nv;
            float q = div_nr32((float)diff, fn, rcp_nr32(fn));
            q = q < -30.0f ? -30.0f : (q > 30.0f ? 30.0f : q);   // finite: no NaN test
            return (double)(c.sign < 0 ? -q : q);
        }
        if constexpr (F32OUT) {
            const float f = __builtin_amdgcn_fmed3f((float)div_nr64((double)diff, c.nv, rcp_nr64(c.nv)), -30.0f, 30.0f);
            return (double)(c.sign < 0 ? -f : f);
        }
        double v = div_nr64((double)diff, c.nv, rcp_nr64(c.nv));
        v = v < -30.0 ? -30.0 : (v > 30.0 ? 30.0 : v);
        return c.sign < 0 ? -v : v;
    }
    if (sizeof(T) == 4 && c.div_f32) {
        // the f32 quotient clipped and negated in f32: the same values as in f64
        // (f32 -> f64 is exact and so are the +-30 clip and the negation)
        // dm_fast: nv in [2^-8, 2^16], |diff| in [2^-90, 2^60]: nothing scaled
        const float fd = (float)diff, fn = (float)c.nv, af = fabsf(fd);
        float q = FAST && c.nv_fast && af >= 0x1p-90f && af <= 0x1p60f ? div_nr32(fd, fn, rcp_nr32(fn))
                                                                                  : fd / fn;
        if (q == q) q = q < -30.0f ? -30.0f : (q > 30.0f ? 30.0f : q);   // np.clip(llr, -30, 30)
        return (double)(c.sign < 0 ? -q : q);
    }
    double v;
    const double dd = (double)diff, ad = fabs(dd);
    // dm_fast: nv in [2^-8, 2^16] (host flag) and |diff| in [2^-900, 2^600]:
    // no operand or quotient the division sequence would scale (zero, whose sign
    // v_div_fixup sets, NaN and inf take the compiler's division)
    if (FAST && c.nv_fast && ad >= 0x1p-900 && ad <= 0x1p600) v = div_nr64(dd, c.nv, rcp_nr64(c.nv));
    else v = dd / c.nv;
    if (v == v) v = v < -30.0 ? -30.0 : (v > 30.0 ? 30.0 : v);
    return c.sign < 0 ? -v : v;
}
template <typename T, bool FAST = false> __device__ __forceinline__ double llr_of(T lo, T hi, const DemapCfg &c) {
    return llr_from_diff<T, FAST>(lo - hi, c);
}

// Square QAM whose label splits into K I-bits and K Q-bits (16/64/256QAM of
// sdr_modem.py:142-220): point (a, q) = levI[a] + j levQ[q].  The minimum of
// numpy's |s - c|^2 over a bit-half is taken at the point nearest in plain
// dx^2 + dy^2 (computed from the same rounded differences) unless two points of
// the half are within a relative 64 ulp of each other: that point is found per
// axis (2^K levels instead of 2^(2K) points) and only the 2*BPS candidates get
// numpy's distance.  Near ties, non-finite input or underflow return false and
// the caller runs the full scan, so the result is the scan's, bit for bit.
//
// The gap test may be stricter than needed, never looser (a stricter test only
// sends more symbols to the exact scan): one tolerance from the largest
// candidate distance serves every half, and once every gap is strictly positive
// the argmin of a half is unique, so min / max order statistics and any
// tie-break give the same candidates.  Inside the fast path every difference is
// finite, so |z| skips numpy's inf / NaN rules (cabs_fin).
// numpy's |z| (npm::cabs_np) for finite re, im: the same operations without the
// inf / NaN selects; f32's square root of fma(r, r, 1) in [1, 2] as the raw
// v_sqrt_f32 plus the compiler's own +-1 ulp correction (its input scaling and
// zero / inf class test are identities on [1, 2]), so bit-identical to sqrtf.
template <typename T> __device__ __forceinline__ T sqrt_1_2(T x) {
    if constexpr (sizeof(T) == 8) {
        return sqrt(x);
    } else {
        const float r = __builtin_amdgcn_sqrtf(x);
        const float dn = __int_as_float(__float_as_int(r) - 1), up = __int_as_float(__float_as_int(r) + 1);
        const float rd = __builtin_fmaf(-dn, r, x), ru = __builtin_fmaf(-up, r, x);
        const float t = rd <= 0.0f ? dn : r;
        return ru > 0.0f ? up : t;
    }
}
template <typename T, bool FAST = false, bool PRE = false> __device__ __forceinline__ T cabs_fin(T re, T im) {
    re = fabs(re);
    im = fabs(im);
    const T larger = re > im ? re : im;
    const T smaller = im < re ? im : re;
    if constexpr (sizeof(T) == 8 && FAST) {
        // larger in [2^-800, 2^800]: no scaling of the denominator; a numerator or
        // quotient small enough to be scaled gives ratio < 2^-169, where
        // fma(ratio, ratio, 1) is 1 whatever its last bits
        if (PRE || (larger >= 0x1p-800 && larger <= 0x1p800)) {
            const double ratio = div_nr64(smaller, larger, rcp_nr64(larger));
            return sqrt_1_2_64(__builtin_fma(ratio, ratio, 1.0)) * larger;
        }
    }
    if constexpr (sizeof(T) == 4 && FAST) {
        // larger in [2^-80, 2^100]: likewise, a scaled numerator or quotient gives
        // ratio < 2^-24 (fma(ratio, ratio, 1) = 1 in f32 below 2^-12.5)
        if (PRE || (larger >= 0x1p-80f && larger <= 0x1p100f)) {
            const float ratio = div_nr32(smaller, larger, rcp_nr32(larger));
            return sqrt_1_2<float>(__builtin_fmaf(ratio, ratio, 1.0f)) * larger;
        }
    }
    const T ratio = larger != (T)0 ? smaller / larger : (T)0;
    return sqrt_1_2<T>(fma(ratio, ratio, (T)1)) * larger;
}

// 16QAM (nv_fast): the per-axis search below for K = 2 in closed
// form, carrying the differences instead of level indices.  Every bit-half holds
// two levels ({0, 1} / {2, 3} for the label's high bit, {0, 2} / {1, 3} for its
// low bit), so its nearest / second nearest / first argmin are a min / max /
// compare of the pair; the axis' nearest is the nearer of the high bit's pair
// minima (ties to the lower labels, as the streamed first-minimum rule) and its
// second nearest min(max of those minima, min of the pair maxima): the same
// values, so the same gap test.  The candidates' differences s - level are the
// ones the search formed (the streamed form forms them again from the indices).
// One range test per symbol replaces the unscaled sequences' per-call tests:
// every candidate's larger |difference| lies between the axes' nearest
// differences and the largest difference, and every LLR numerator below twice
// its square; a symbol outside declines (its LLRs come from the full chain).
template <typename T, bool F32OUT = false>
__device__ __forceinline__ bool sym_llrs_pairs16(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[4]) {
    constexpr bool F32 = sizeof(T) == 4;
    if (!(isfinite(sr) && isfinite(si))) return false;
    const T *lev_i = cons + 2 * 16, *lev_q = lev_i + 4;
    const T inf = (T)INFINITY;
    const T eps = F32 ? (T)3.8e-6 : (T)7.2e-15, tau = F32 ? (T)1e-30 : (T)1e-290;
    T dn[2], dc[2][2], all1[2];
    bool vn[2][2];
    T gap = inf, top = (T)0, hi = (T)0, dmax = (T)0;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        const T s = ax ? si : sr;
        const T *lev = ax ? lev_q : lev_i;
        T d[4], d2[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            d[a] = s - lev[a];
            d2[a] = d[a] * d[a];
            dmax = fmax(dmax, fabs(d[a]));
        }
        T b1[2][2], b2[2][2], bd[2][2];
        bool lt[2][2];
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const int p = b ? v : 2 * v, q = b ? v + 2 : 2 * v + 1;   // the half's two levels, p < q
                lt[b][v] = d2[q] < d2[p];
                b1[b][v] = fmin(d2[p], d2[q]);
                b2[b][v] = fmax(d2[p], d2[q]);
                bd[b][v] = lt[b][v] ? d[q] : d[p];
                gap = fmin(gap, b2[b][v] - b1[b][v]);
                top = fmax(top, b1[b][v]);
                hi = fmax(hi, b2[b][v]);
            }
        const T a1 = fmin(b1[0][0], b1[0][1]), a2 = fmin(fmax(b1[0][0], b1[0][1]), fmin(b2[0][0], b2[0][1]));
        gap = fmin(gap, a2 - a1);
        hi = fmax(hi, a2);
        all1[ax] = a1;
        const bool hv = b1[0][1] < b1[0][0];                 // the nearest level's label bits
        const bool lv = hv ? lt[0][1] : lt[0][0];
        dn[ax] = hv ? bd[0][1] : bd[0][0];
        dc[ax][0] = hv ? bd[0][0] : bd[0][1];               // nearest with the other high bit
        dc[ax][1] = lv ? bd[1][0] : bd[1][1];               // nearest with the other low bit
        vn[ax][0] = hv;
        vn[ax][1] = lv;
    }
    const T tol = eps * (top + fmax(all1[0], all1[1])) + tau;
    const T l0 = fmax(fabs(dn[0]), fabs(dn[1]));
    if (!(hi < inf && gap > tol && l0 >= (F32 ? (T)0x1p-80f : (T)0x1p-800) && dmax <= (F32 ? (T)0x1p29f : (T)0x1p290)))
        return false;
    const T an = cabs_fin<T, true, true>(dn[0], dn[1]);
    const T dq = an * an;
    const T lo = F32 ? (c.div_f32 ? (T)0x1p-90f : (T)0x1p-149f) : (T)0x1p-900;
    T diff[4];
#pragma unroll
    for (int ax = 0; ax < 2; ++ax)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const T a = ax ? cabs_fin<T, true, true>(dn[0], dc[1][b]) : cabs_fin<T, true, true>(dc[0][b], dn[1]);
            const T ao = a * a;
            diff[ax * 2 + b] = vn[ax][b] ? ao - dq : dq - ao;   // m[0] - m[1], m[vn] = dn
        }
    if (!(fmin(fmin(fabs(diff[0]), fabs(diff[1])), fmin(fabs(diff[2]), fabs(diff[3]))) >= lo)) return false;
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = llr_from_diff<T, true, true, F32OUT>(diff[k], c);
    return true;
}

template <typename T, int BPS, bool F32OUT = false>
__device__ __forceinline__ bool sym_llrs_sep(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    constexpr int K = BPS / 2, L = 1 << K;
    const T *lev_i = cons + 2 * (1 << BPS), *lev_q = lev_i + L;
    const T inf = (T)INFINITY;
    const T eps = sizeof(T) == 4 ? (T)3.8e-6 : (T)7.2e-15, tau = sizeof(T) == 4 ? (T)1e-30 : (T)1e-290;
    if constexpr (K == 2 && dm_fast(BPS)) {
        if (c.nv_fast) return sym_llrs_pairs16<T, F32OUT>(sr, si, cons, c, out);
    }
    T all1[2], all2[2], b1[2][K][2], b2[2][K][2];   // nearest / second nearest: axis, bit-halves
    int arg[2][K][2], allarg[2];
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        const T s = ax ? si : sr;
        const T *lev = ax ? lev_q : lev_i;
        // streamed over the levels: nearest / second nearest of the axis and of
        // each bit-half (a NaN distance is dropped by fmin / fmax; then every
        // distance of the axis is NaN, the minima stay inf and the test below
        // fails)
        T m1 = inf, m2 = inf;
        int am = 0;
#pragma unroll
        for (int b = 0; b < K; ++b)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                b1[ax][b][v] = b2[ax][b][v] = inf;
                arg[ax][b][v] = 0;
            }
#pragma unroll
        for (int a = 0; a < L; ++a) {
            const T d = s - lev[a];
            const T d2 = d * d;
            m2 = fmin(m2, fmax(m1, d2));
            am = d2 < m1 ? a : am;
            m1 = fmin(m1, d2);
#pragma unroll
            for (int b = 0; b < K; ++b) {
                const int v = (a >> (K - 1 - b)) & 1;
                b2[ax][b][v] = fmin(b2[ax][b][v], fmax(b1[ax][b][v], d2));
                arg[ax][b][v] = d2 < b1[ax][b][v] ? a : arg[ax][b][v];
                b1[ax][b][v] = fmin(b1[ax][b][v], d2);
            }
        }
        all1[ax] = m1;
        all2[ax] = m2;
        allarg[ax] = am;
    }
    T gap = fmin(all2[0] - all1[0], all2[1] - all1[1]), top = (T)0, hi = fmax(all2[0], all2[1]);
#pragma unroll
    for (int ax = 0; ax < 2; ++ax)
#pragma unroll
        for (int b = 0; b < K; ++b)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                gap = fmin(gap, b2[ax][b][v] - b1[ax][b][v]);
                top = fmax(top, b1[ax][b][v]);
                hi = fmax(hi, b2[ax][b][v]);
            }
    // every gap above the tolerance of the largest candidate distance
    // (best + the other axis' nearest), every second nearest finite
    const T tol = eps * (top + fmax(all1[0], all1[1])) + tau;
    if (!(hi < inf && gap > tol)) return false;
    // The half holding the overall nearest point has that point as its
    // candidate, so its distance is shared by every bit: BPS + 1 numpy
    // distances instead of 2 * BPS.
    const T an = cabs_fin<T, dm_fast(BPS)>(sr - lev_i[allarg[0]], si - lev_q[allarg[1]]);
    const T dn = an * an;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax)
#pragma unroll
        for (int b = 0; b < K; ++b) {
            const int vn = (allarg[ax] >> (K - 1 - b)) & 1, vo = vn ^ 1;
            const int ia = ax ? allarg[0] : arg[0][b][vo], iq = ax ? arg[1][b][vo] : allarg[1];
            const T a = cabs_fin<T, dm_fast(BPS)>(sr - lev_i[ia], si - lev_q[iq]);
            const T ao = a * a;
            out[ax * K + b] = llr_from_diff<T, dm_fast(BPS)>(vn ? ao - dn : dn - ao, c);   // m[0] - m[1], m[vn] = dn
        }
    return true;
}

// All BPS LLRs of one symbol, reference sign (positive -> bit 1) unless
// c.sign < 0.  Streams over the M points keeping a running min per bit and
// label value, so no distance array is materialised.
template <typename T, int BPS, bool FIN, int M = (1 << BPS), int UNROLL = (M <= 16 ? M : 8)>
__device__ __forceinline__ void sym_llrs_scan(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    T m0[BPS], m1[BPS];
    bool n0[BPS], n1[BPS];
#pragma unroll
    for (int b = 0; b < BPS; ++b) {
        m0[b] = m1[b] = (T)INFINITY;
        n0[b] = n1[b] = false;
    }
    // M is the full label space; a table with fewer points (c.M < M) stops early.
#pragma unroll UNROLL
    for (int m = 0; m < M; ++m) {
        if (M > 2 && m >= c.M) break;
        const T a = FIN ? cabs_fin<T, dm_fast(BPS)>(sr - cons[2 * m], si - cons[2 * m + 1]) : cabs_np<T>(sr - cons[2 * m], si - cons[2 * m + 1]);
        const T v = a * a;                     // np.abs(s - constellation) ** 2
        const bool vn = v != v;
#pragma unroll
        for (int b = 0; b < BPS; ++b) {
            if ((m >> (BPS - 1 - b)) & 1) {
                n1[b] |= vn;
                m1[b] = v < m1[b] ? v : m1[b];
            } else {
                n0[b] |= vn;
                m0[b] = v < m0[b] ? v : m0[b];
            }
        }
    }
#pragma unroll
    for (int b = 0; b < BPS; ++b)
        out[b] = llr_of<T, dm_fast(BPS)>(n0[b] ? (T)NAN : m0[b], n1[b] ? (T)NAN : m1[b], c);   // np.min propagates NaN
}

// sym_llrs_scan_pre (BPSK / QPSK / 8PSK, finite symbols): the scan with the
// unscaled division / square root under one range test per symbol instead of one
// per point (sym_llrs_pairs16): every point's larger |difference| within [2^-80,
// 2^29] (f32) / [2^-800, 2^290] (f64) and nv_fast, for every lane of the wave, or
// false and the caller scans with the per-point tests.  Finite differences below
// 2^29 give finite squares, so np.min's NaN rule never applies; an LLR numerator
// of zero or below the quotient's range takes the compiler's division (its sign of
// zero), per lane.  Measured (profiles/r05/demap_scan/, same planes): 8PSK
// 12.66 -> 11.61 ms, QPSK 5.88 -> 5.70 ms per 1 M codewords.
// The plane kernels take the LLRs' f32 form (llr_from_diff F32OUT = DM_F32OUT):
// same planes, 16QAM 12.62 -> 12.29 ms, 256QAM 12.82 -> 12.30, 8PSK 11.27 -> 11.11 per
// 1 M codewords (profiles/r05/demap_f32out/)
constexpr bool DM_F32OUT = true;
template <typename T, int BPS, bool F32OUT = false, int M = (1 << BPS)>
__device__ __forceinline__ bool sym_llrs_scan_pre(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    constexpr bool F32 = sizeof(T) == 4;
    T dx[M], dy[M], lmin = (T)INFINITY, lmax = (T)0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const bool on = M <= 2 || m < c.M;   // a table with fewer points than 2^BPS
        dx[m] = sr - cons[2 * m];
        dy[m] = si - cons[2 * m + 1];
        const T l = fmax(fabs(dx[m]), fabs(dy[m]));
        lmin = on ? fmin(lmin, l) : lmin;
        lmax = on ? fmax(lmax, l) : lmax;
    }
    const bool ok = c.nv_fast && lmin >= (F32 ? (T)0x1p-80f : (T)0x1p-800) && lmax <= (F32 ? (T)0x1p29f : (T)0x1p290);
    if (!__all(ok)) return false;
    T m0[BPS], m1[BPS];
#pragma unroll
    for (int b = 0; b < BPS; ++b) m0[b] = m1[b] = (T)INFINITY;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        if (M > 2 && m >= c.M) break;
        const T a = cabs_fin<T, true, true>(dx[m], dy[m]);
        const T v = a * a;                     // np.abs(s - constellation) ** 2
#pragma unroll
        for (int b = 0; b < BPS; ++b) {
            if ((m >> (BPS - 1 - b)) & 1) m1[b] = v < m1[b] ? v : m1[b];
            else m0[b] = v < m0[b] ? v : m0[b];
        }
    }
    const T lo = F32 ? (c.div_f32 ? (T)0x1p-90f : (T)0x1p-149f) : (T)0x1p-900;
#pragma unroll
    for (int b = 0; b < BPS; ++b) {
        const T d = m0[b] - m1[b];
        if (fabs(d) >= lo) out[b] = llr_from_diff<T, true, true, F32OUT>(d, c);
        else out[b] = llr_from_diff<T, false>(d, c);
    }
    return true;
}

// With every lane's symbol finite (the table is), every difference is finite
// and |z| is cabs_fin; BPSK / QPSK / 8PSK (M <= 8, the scan is their only
// path) take that copy when the whole wave qualifies.
template <typename T, int BPS, bool F32OUT = false, int M = (1 << BPS)>
__device__ __forceinline__ void sym_llrs(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    if constexpr (M <= 8) {
        if (__all(isfinite(sr) && isfinite(si))) {
            if constexpr (dm_fast(BPS)) {
                if (sym_llrs_scan_pre<T, BPS, F32OUT>(sr, si, cons, c, out)) return;
            }
            sym_llrs_scan<T, BPS, true>(sr, si, cons, c, out);
            return;
        }
    }
    sym_llrs_scan<T, BPS, false>(sr, si, cons, c, out);
}

// 256QAM (K = 4) keeps the previous form of the same search (per-half best and
// second by compare-select, numpy's |z| with its inf / NaN rules): the form
// above compiles to 198-230 VGPRs at K = 4 (2 waves per SIMD, 70.6 -> 100.8 ms
// per 1 M codewords) against 135; at K = 2 / 3 it is 12 % faster.
template <typename T, int BPS>
__device__ __forceinline__ bool sym_llrs_sep_seq(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    constexpr int K = BPS / 2, L = 1 << K;
    const T *lev_i = cons + 2 * (1 << BPS), *lev_q = lev_i + L;
    const T inf = (T)INFINITY;
    const T eps = sizeof(T) == 4 ? (T)3.8e-6 : (T)7.2e-15, tau = sizeof(T) == 4 ? (T)1e-30 : (T)1e-290;
    T best[2][K][2], second[2][K][2], all1[2], all2[2];
    int arg[2][K][2], allarg[2];
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        const T s = ax ? si : sr;
        const T *lev = ax ? lev_q : lev_i;
        all1[ax] = all2[ax] = inf;
        allarg[ax] = 0;
#pragma unroll
        for (int b = 0; b < K; ++b)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                best[ax][b][v] = second[ax][b][v] = inf;
                arg[ax][b][v] = 0;
            }
#pragma unroll
        for (int a = 0; a < L; ++a) {
            const T d = s - lev[a];
            const T d2 = d * d;
            all2[ax] = d2 < all1[ax] ? all1[ax] : (d2 < all2[ax] ? d2 : all2[ax]);
            allarg[ax] = d2 < all1[ax] ? a : allarg[ax];
            all1[ax] = d2 < all1[ax] ? d2 : all1[ax];
#pragma unroll
            for (int b = 0; b < K; ++b) {
                const int v = (a >> (K - 1 - b)) & 1;
                T &b1 = best[ax][b][v], &b2 = second[ax][b][v];
                b2 = d2 < b1 ? b1 : (d2 < b2 ? d2 : b2);
                arg[ax][b][v] = d2 < b1 ? a : arg[ax][b][v];
                b1 = d2 < b1 ? d2 : b1;
            }
        }
    }
    bool ok = all2[0] < inf && all2[1] < inf;   // every value finite (NaN compares false)
#pragma unroll
    for (int ax = 0; ax < 2; ++ax)
#pragma unroll
        for (int b = 0; b < K; ++b)
#pragma unroll
            for (int v = 0; v < 2; ++v) {
                const T e = best[ax][b][v] + all1[ax ^ 1];                  // the half's nearest point
                const T tol = eps * e + tau;
                ok = ok && second[ax][b][v] < inf && second[ax][b][v] - best[ax][b][v] > tol &&
                     all2[ax ^ 1] - all1[ax ^ 1] > tol;
            }
    if (!ok) return false;
    // The half holding the overall nearest point has that point as its
    // candidate (same first-minimum rule per axis), so its distance is shared
    // by every bit: BPS + 1 numpy distances instead of 2 * BPS.
    const T an = cabs_fin<T, dm_fast(BPS)>(sr - lev_i[allarg[0]], si - lev_q[allarg[1]]);
    const T dn = an * an;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax)
#pragma unroll
        for (int b = 0; b < K; ++b) {
            const int vn = (allarg[ax] >> (K - 1 - b)) & 1, vo = vn ^ 1;
            const int ia = ax ? allarg[0] : arg[0][b][vo], iq = ax ? arg[1][b][vo] : allarg[1];
            const T a = cabs_fin<T, dm_fast(BPS)>(sr - lev_i[ia], si - lev_q[iq]);
            const T ao = a * a;
            out[ax * K + b] = llr_from_diff<T, dm_fast(BPS)>(vn ? ao - dn : dn - ao, c);   // m[0] - m[1], m[vn] = dn
        }
    return true;
}

// Uniform PAM on each axis with the reference's labelling (sep == 2, detected on
// the host: the 16/64/256QAM tables of sdr_modem.py:142-207 and
// test_sdr_with_coding.py:72-86 put label a at level position gray[a] = a ^ (a >> 1),
// so the label at position p is the inverse Gray code of p -- adjacent levels can
// differ in several label bits).  The same candidates as the searches above, found
// without scanning the 2^K levels: the nearest level position p from
// (s - x_0) / delta, validated by the gap to both neighbours; for label bit b the
// positions with the other bit value nearest to s are the first such position left
// of p and the first right of p (host table nb[b][p] = {left, right}, -1 / L when
// none): every other one lies farther on the same side, since distance grows
// away from s by at least delta^2 per position.  With every decisive gap above the
// tolerance of the largest candidate distance, the argmin of numpy's |s - c|^2 over
// each bit-half is unique and is the candidate, so the LLRs are the full scan's bit
// for bit; anything else (non-finite input, near ties, a wrong position estimate)
// returns false and the caller scans.
__device__ __forceinline__ int gray_inv(int q, int K) {
    int a = q;
    for (int sh = 1; sh < K; ++sh) a ^= q >> sh;
    return a;
}
template <typename T, int BPS, bool F32OUT = false>
__device__ __forceinline__ bool sym_llrs_gray(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    constexpr int K = BPS / 2, L = 1 << K;
    if (!(isfinite(sr) && isfinite(si))) return false;
    const T *pos_i = cons + 2 * (1 << BPS) + 2 * L, *pos_q = pos_i + L, *prm = pos_q + L, *nb = prm + 4;
    const T inf = (T)INFINITY;
    const T eps = sizeof(T) == 4 ? (T)3.8e-6 : (T)7.2e-15, tau = sizeof(T) == 4 ? (T)1e-30 : (T)1e-290;
    int p[2], cb[2][K];
    T e0s[2], cds[2][K];   // the nearest level's and the candidates' differences s - level
    T gapmin = inf, dmax = (T)0;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        const T s = ax ? si : sr;
        const T *pos = ax ? pos_q : pos_i;
        const T t = fmin(fmax(rint((s - prm[2 * ax]) * prm[2 * ax + 1]), (T)0), (T)(L - 1));
        const int q = (int)t;
        const T e0 = s - pos[q], d0 = e0 * e0;
        e0s[ax] = e0;
        const T el = s - pos[q > 0 ? q - 1 : q], er = s - pos[q < L - 1 ? q + 1 : q];
        const T dl = q > 0 ? el * el : inf, dr = q < L - 1 ? er * er : inf;
        gapmin = fmin(gapmin, fmin(dl, dr) - d0);
        dmax = fmax(dmax, fmax(d0, fmax(q > 0 ? dl : (T)0, q < L - 1 ? dr : (T)0)));
#pragma unroll
        for (int b = 0; b < K; ++b) {
            const int lc = (int)nb[(b * L + q) * 2], rc = (int)nb[(b * L + q) * 2 + 1];
            const bool lv = lc >= 0, rv = rc < L;
            const T xl = s - pos[lv ? lc : q], xr = s - pos[rv ? rc : q];
            const T dL = lv ? xl * xl : inf, dR = rv ? xr * xr : inf;
            if (lv && rv) gapmin = fmin(gapmin, fabs(dL - dR));
            cb[ax][b] = dL <= dR ? lc : rc;
            cds[ax][b] = dL <= dR ? xl : xr;
            dmax = fmax(dmax, fmax(lv ? dL : (T)0, rv ? dR : (T)0));
        }
        p[ax] = q;
    }
    const T tol = eps * (2 * dmax) + tau;
    if (!(dmax < inf && gapmin > tol)) return false;
    // (a noise variance outside [2^-8, 2^16] declines every symbol to the
    // callers' other searches: the compiler's sequences would hold their
    // registers in this kernel too, a step of occupancy)
    if (!c.nv_fast) return false;
    // the differences the search formed, and one range test per symbol for the
    // unscaled division / square root (sym_llrs_pairs16): every candidate's larger
    // |difference| lies between the axes' nearest differences and sqrt(dmax);
    // outside, or an LLR numerator below the quotient's range, the symbol declines
    // to the full chain
    constexpr bool F32 = sizeof(T) == 4;
    const T l0 = fmax(fabs(e0s[0]), fabs(e0s[1]));
    if (!(l0 >= (F32 ? (T)0x1p-80f : (T)0x1p-800) && dmax <= (F32 ? (T)0x1p58f : (T)0x1p580))) return false;
    const T an = cabs_fin<T, true, true>(e0s[0], e0s[1]);
    const T dq = an * an;
    const T lo = F32 ? (c.div_f32 ? (T)0x1p-90f : (T)0x1p-149f) : (T)0x1p-900;
    T diff[BPS], dlo = inf;
#pragma unroll
    for (int ax = 0; ax < 2; ++ax) {
        const int lab = gray_inv(p[ax], K);
#pragma unroll
        for (int b = 0; b < K; ++b) {
            const int vn = (lab >> (K - 1 - b)) & 1;
            const T a = ax ? cabs_fin<T, true, true>(e0s[0], cds[1][b]) : cabs_fin<T, true, true>(cds[0][b], e0s[1]);
            const T ao = a * a;
            diff[ax * K + b] = vn ? ao - dq : dq - ao;   // m[0] - m[1], m[vn] = dn
            dlo = fmin(dlo, fabs(diff[ax * K + b]));
        }
    }
    if (!(dlo >= lo)) return false;
#pragma unroll
    for (int k = 0; k < BPS; ++k) out[k] = llr_from_diff<T, true, true, F32OUT>(diff[k], c);
    return true;
}

// TDEC_DM_STATS (measurement build): symbols per demap path, read by
// tdec_demap_stats: [0] symbols, [1] taken by the Gray search, [2] by the
// per-axis searches, [3] by the full scan, [4] the table's sep class of the last
// symbol (+1)
#ifndef TDEC_DM_STATS
#define TDEC_DM_STATS 0
#endif
#if TDEC_DM_STATS
__device__ unsigned long long g_dm_stats[8];
__device__ __forceinline__ void dm_count(int path, int sep) {
    atomicAdd(&g_dm_stats[0], 1ull);
    atomicAdd(&g_dm_stats[path], 1ull);
    g_dm_stats[4] = (unsigned long long)(sep + 1);
}
#else
__device__ __forceinline__ void dm_count(int, int) {}
#endif
template <typename T, int BPS, bool F32OUT = false>
__device__ __forceinline__ void demap_sym(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    // 64 / 256QAM (measured, 1 M codewords, same planes: 20.2 -> 17.6 ms, 70.3 -> 56.2 ms);
    // 16QAM's 4-level scan is cheaper than the table lookups (14.9 vs 16.0 ms)
    if constexpr (BPS >= 6 && BPS % 2 == 0) {
        if (c.sep == 2 && sym_llrs_gray<T, BPS, F32OUT>(sr, si, cons, c, out)) return dm_count(1, c.sep);
    }
    if constexpr (BPS >= 8 && BPS % 2 == 0) {
        if (c.sep && sym_llrs_sep_seq<T, BPS>(sr, si, cons, c, out)) return dm_count(2, c.sep);
    } else if constexpr (BPS >= 4 && BPS % 2 == 0) {
        if (c.sep && sym_llrs_sep<T, BPS, F32OUT>(sr, si, cons, c, out)) return dm_count(2, c.sep);
    }
    sym_llrs<T, BPS, F32OUT>(sr, si, cons, c, out);
    dm_count(3, c.sep);
}

// The table (and a separable table's axis levels) into LDS.
template <typename T, int BPS> __device__ __forceinline__ void load_table(T *cons, const T *cons_g, const DemapCfg &c) {
    constexpr int L = 1 << (BPS / 2);
    const int n = 2 * c.M + (c.sep ? 2 * L : 0) + (c.sep == 2 ? 2 * L + 4 + 2 * (BPS / 2) * L : 0);
    for (int i = threadIdx.x; i < n; i += BLOCK) cons[i] = cons_g[i];
}

template <typename T, typename S, int BPS>
__global__ __launch_bounds__(BLOCK) void k_demap(const S *syms, long n_sym, const T *cons_g, DemapCfg c, double *llr) {
    __shared__ T cons[DM_TAB];
    load_table<T, BPS>(cons, cons_g, c);
    __syncthreads();
    const long s = (long)blockIdx.x * BLOCK + threadIdx.x;
    if (s >= n_sym) return;
    double v[BPS];
    demap_sym<T, BPS>((T)syms[2 * s], (T)syms[2 * s + 1], cons, c, v);
#pragma unroll
    for (int b = 0; b < BPS; ++b) llr[s * BPS + b] = v[b];
}

// ---- self-tests of the demapper's exact shortcuts (tdec_selftest) -------------------
// which 0: sqrt_1_2 against sqrtf and against the correctly rounded f64 square
// root rounded to f32 (innocuous double rounding for sqrt) for every f32 in
// [1, 2]; which 1 / 2: cabs_fin against npm::cabs_np (f32 / f64) on n
// splitmix64 bit patterns taken as finite (re, im) pairs, every exponent.
// bad[0] counts differing results, bad[1] the items evaluated.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ __launch_bounds__(BLOCK) void k_selftest(int which, long long n, unsigned long long seed,
                                                    unsigned long long *bad) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    bool ok = true;
    if (which == 0) {
        const float x = __uint_as_float(0x3F800000u + (unsigned)i);
        const unsigned a = __float_as_uint(sqrt_1_2<float>(x));
        ok = a == __float_as_uint(sqrtf(x)) && a == __float_as_uint((float)sqrt((double)x));
    } else if (which == 1) {
        const unsigned long long r = splitmix64(seed + 2 * (unsigned long long)i);
        float re = __uint_as_float((unsigned)r), im = __uint_as_float((unsigned)(r >> 32));
        if (!isfinite(re)) re = 1.5f;
        if (!isfinite(im)) im = -0.75f;
        ok = __float_as_uint(cabs_fin<float>(re, im)) == __float_as_uint(cabs_np<float>(re, im)) &&
             __float_as_uint(cabs_fin<float, true>(re, im)) == __float_as_uint(cabs_np<float>(re, im));
    } else if (which == 3) {
        // log-MAP primitives outside the captured tables: every f32 t >= 48 (bit
        // patterns 0x42400000 .. 0x7F800000 = +inf, n ignored) gives 0 <= 2^-t <= 2^-39
        // (256 * 2^-t is absorbed by any sum >= 1 - 2^-23), with 2^-inf = +0; item 0 also
        // checks NaN -> NaN for both instructions and log2(1) = 0.
        const float t = __uint_as_float(0x42400000u + (unsigned)i);
        const float e = hw_exp2(-t);
        ok = e >= 0.0f && e <= 0x1p-39f && (t != INFINITY || __float_as_uint(e) == 0u);
        if (i == 0) {
            const float qn = __uint_as_float(0x7FC00000u);
            ok = ok && hw_exp2(qn) != hw_exp2(qn) && hw_log2(qn) != hw_log2(qn) && __float_as_uint(hw_log2(1.0f)) == 0u;
        }
    } else if (which == 4) {
        // the unscaled sequences (dm_fast) against the compiler's on the demapper's ranges:
        // |z| of (re, im) with exponents in [-64, 16) (a quarter of the items with
        // |im| within a factor 2 of |re|); a / b with |a| in [2^-900, 2^600), b in
        // [2^-8, 2^100); sqrt on [1, 2)
        const unsigned long long r0 = splitmix64(seed + 4 * (unsigned long long)i), r1 = splitmix64(r0),
                                 r2 = splitmix64(r1), r3 = splitmix64(r2);
        auto mk = [](unsigned long long r, int e) {   // random sign and mantissa, exponent e
            return __longlong_as_double((long long)((r & 0x800FFFFFFFFFFFFFull) | ((unsigned long long)(e + 1023) << 52)));
        };
        const int ea = (int)(r2 % 80) - 64;
        const int eb = (r2 >> 8) & 3 ? (int)((r2 >> 16) % 80) - 64 : ea + (int)((r2 >> 24) & 1);
        const double re = mk(r0, ea), im = mk(r1, eb);
        ok = __double_as_longlong(cabs_fin<double, true>(re, im)) == __double_as_longlong(cabs_np<double>(re, im));
        const double a = mk(r0, (int)(r3 % 1500) - 900), b = fabs(mk(r1, (int)((r3 >> 16) % 108) - 8));
        ok = ok && __double_as_longlong(div_nr64(a, b, rcp_nr64(b))) == __double_as_longlong(a / b);
        const double x = __longlong_as_double((long long)((r2 & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull));
        ok = ok && __double_as_longlong(sqrt_1_2_64(x)) == __double_as_longlong(sqrt(x));
        // f32: |z| with exponents in [-64, 16), a / b with |a| in [2^-90, 2^60), b in [2^-8, 2^16)
        auto mkf = [](unsigned r, int e) { return __uint_as_float((r & 0x807FFFFFu) | ((unsigned)(e + 127) << 23)); };
        const float fre = mkf((unsigned)r0, ea), fim = mkf((unsigned)(r0 >> 32), eb);
        ok = ok && __float_as_uint(cabs_fin<float, true>(fre, fim)) == __float_as_uint(cabs_np<float>(fre, fim));
        const float fa = mkf((unsigned)r1, (int)(r3 % 150) - 90), fb = fabsf(mkf((unsigned)(r1 >> 32), (int)((r3 >> 16) % 24) - 8));
        ok = ok && __float_as_uint(div_nr32(fa, fb, rcp_nr32(fb))) == __float_as_uint(fa / fb);
    } else {
        double re = __longlong_as_double((long long)splitmix64(seed + 2 * (unsigned long long)i));
        double im = __longlong_as_double((long long)splitmix64(seed + 2 * (unsigned long long)i + 1));
        if (!isfinite(re)) re = 1.5;
        if (!isfinite(im)) im = -0.75;
        ok = __double_as_longlong(cabs_fin<double>(re, im)) == __double_as_longlong(cabs_np<double>(re, im)) &&
             __double_as_longlong(cabs_fin<double, true>(re, im)) == __double_as_longlong(cabs_np<double>(re, im));
    }
    if (!ok) atomicAdd(bad, 1ull);
    const unsigned long long act = __ballot(1);   // bad[1]: items evaluated (a launch that did not run fails)
    if ((threadIdx.x & (WAVE - 1)) == (unsigned)__ffsll((long long)act) - 1) atomicAdd(bad + 1, (unsigned long long)__popcll(act));
}

// The log-MAP primitives' exact outputs (test infrastructure: the oracle's
// tables, oracle/tdec_oracle.c orc_set_trans): out[i] = v_exp_f32(-t) (which 0)
// or v_log_f32(w) (which 1) of the f32 whose bit pattern is lo + i.
__global__ __launch_bounds__(BLOCK) void k_trans_table(int which, unsigned lo, long long n, float *out) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const float x = __uint_as_float(lo + (unsigned)i);
    out[i] = which == 0 ? hw_exp2(-x) : hw_log2(x);
}

// Fused demap -> f32 -> de-puncture planes (the bench path).
// One item = one 64-codeword tile x DM_KC trellis steps (one block per item).
// Phase 1: the block's threads demap every symbol covering the LLR range of those
// steps (couples consume LLRs in order, so the range is contiguous) into an LDS
// tile, decoder sign, rounded to f32 as decode() does (:466).  Phase 2: each
// thread assembles whole plane entries X[k] = {A, B, W1, Y1} (float4), Z[k] =
// {W2, Y2} (float2) and stores them coalesced; punctured or missing LLRs are 0.0
// (:469-474; the harness pads to n_coded, test_sdr_with_coding.py:474-478).
// src[c*N + k] = LLR index of plane component c (X.xyzw, -, -, Z.xy) or -1;
// off[k] = first LLR index of couple k (off[N] = n_llr).
// Split tables (round 4, square 16 / 64 / 256QAM): k_demap_planes runs only the
// fast exact search (the Gray positions for 64 / 256QAM, the per-axis search for
// 16QAM) and appends the symbols it declines (near ties, non-finite input, a
// non-separable table: 0.02-0.08 % of them at 2 dB) to a list in HBM; k_demap_fix
// then gives those the rest of demap_sym's chain and overwrites their plane
// entries.  The fallbacks' registers (256QAM: 148 VGPRs and 311 SGPR spills with
// them inline, three waves per SIMD) are then not the main kernel's.  A tile whose
// declines overflow the list is flagged and k_demap_fix redoes all of its symbols.
// Same planes: every path returns the scan's LLRs.  (The fallback in a second loop
// of the same kernel kept the registers and was 2.3x slower on 256QAM,
// profiles/r04e/ab_demap_*; a persistent grid, one wave per 16 codewords, and the
// other forms in the DESIGN.md appendix measured slower.)
// KC: couples per block (its LDS tile [64][6 * KC + 2 * BPS + 1] f32 bounds the
// blocks per CU: 16 -> 27-29 KB, five).  QPSK's kernel is LDS-bound at five blocks
// per CU and its work per block small: 12 couples measured faster (5.47 vs 5.82 ms
// per 1 M N = 212 codewords); 16QAM slower with 12 or 8 (13.45 / 13.41 vs 12.75 ms,
// profiles/r05/demap_kc/).
constexpr int DM_KC = 16;                  // couples per block
constexpr int DM_MAXL = DM_KC * 6;         // max LLRs per chunk (6 per couple at rate 1/3)
__host__ __device__ constexpr int dm_kc(int bps) { return bps == 2 ? 12 : DM_KC; }
__host__ __device__ constexpr bool dm_split(int bps) { return bps >= 4 && bps % 2 == 0; }

// The decline list of k_demap_planes (split tables): entries {codeword, symbol},
// the entry count, and per-tile overflow flags.
constexpr unsigned DM_DECL_CAP = 1u << 21;   // entries (16 MiB): 4x the declines of 1 M 256QAM codewords at 2 dB
// A table takes the split path when its fast search can accept its symbols: the
// Gray search (64 / 256QAM) needs sep == 2, 16QAM's per-axis search sep >= 1;
// any other table would decline every symbol.
__host__ __device__ constexpr bool dm_split_table(int bps, int sep) {
    return dm_split(bps) && (bps >= 6 ? sep == 2 : sep >= 1);
}
struct DemapDecl {
    int2 *list;
    unsigned *count;
    unsigned char *ovf;
    unsigned cap;
};

// the fast exact search of a split table; false: declined
template <typename T, int BPS, bool F32OUT = false>
__device__ __forceinline__ bool demap_fast(T sr, T si, const T *cons, const DemapCfg &c, double (&out)[BPS]) {
    if constexpr (BPS >= 6) return c.sep == 2 && sym_llrs_gray<T, BPS, F32OUT>(sr, si, cons, c, out);
    else return c.sep && sym_llrs_sep<T, BPS, F32OUT>(sr, si, cons, c, out);
}

template <typename T, int BPS, bool SPLIT = false>
__global__ __launch_bounds__(BLOCK) void k_demap_planes(int B, int N, int S, const float *syms, const T *cons_g,
                                                       DemapCfg c, const int *__restrict__ src,
                                                       const int *__restrict__ off, long n_avail, float *planes,
                                                       long n_items, DemapDecl dd) {
    __shared__ T cons[DM_TAB];
    // couples per item, LDS row stride (odd); the tile by label bit (column b * ns +
    // symbol: the 64 lanes of a phase-1 store hit 64 banks, 1.5-4 % faster on every
    // table, profiles/r05/demap_planar/) with room for the item's straddling symbols
    constexpr int KC = dm_kc(BPS), LD = 6 * KC + 2 * BPS + 1;
    __shared__ float L[WAVE * LD];
    static_assert(!SPLIT || dm_split(BPS), "split only for square 16 / 64 / 256QAM");
    const int me = (int)threadIdx.x & (WAVE - 1);
    load_table<T, BPS>(cons, cons_g, c);
    const int chunks = (N + KC - 1) / KC;
    __syncthreads();
    for (long item = blockIdx.x; item < n_items; item += gridDim.x) {
        const long tile = item / chunks;
        const int k0 = (int)(item % chunks) * KC;
        const int k1 = min(N, k0 + KC);
        const long j0 = off[k0], j1 = off[k1];
        const long s0 = j0 / BPS, s1 = (j1 + BPS - 1) / BPS;        // symbols covering [j0, j1)
        const int ns = (int)(s1 - s0);
        // item t = (lane, si), consecutive threads: consecutive symbols; the
        // quotient and remainder of t by ns advance by those of BLOCK each step
        const int T0 = (int)threadIdx.x;
        const int dq = BLOCK / ns, dr = BLOCK - dq * ns;
        int lane = T0 / ns, si = T0 - lane * ns;
        const int nt = WAVE * ns;
        // the symbol of item t (lane ln, symbol sx), zero past the batch / the item's end
        auto sym_at = [&](int t, int ln, int sx) -> float2 {
            const long cw = tile * WAVE + ln, s = s0 + sx;
            return t < nt && cw < B && s < S ? *reinterpret_cast<const float2 *>(syms + 2 * (cw * S + s))
                                             : make_float2(0.0f, 0.0f);
        };
        // the next item's symbol is loaded before this one is demapped (8PSK / 16QAM:
        // measured faster; QPSK and 64 / 256QAM slower)
        constexpr bool PF = BPS == 3 || BPS == 4;
        float2 zn = PF ? sym_at(T0, lane, si) : make_float2(0.0f, 0.0f);
        for (int t = T0; t < nt; t += BLOCK) {
            const int ln = lane, sx = si;
            lane += dq;
            si += dr;
            if (si >= ns) {
                si -= ns;
                ++lane;
            }
            const float2 zc = PF ? zn : sym_at(t, ln, sx);
            if (PF) zn = sym_at(t + BLOCK, lane, si);
            const long cw = tile * WAVE + ln;
            const long s = s0 + sx;
            const bool live = cw < B && s < S;
            double v[BPS];
            if constexpr (SPLIT) {
                bool dec = false;
                if (live) dec = !demap_fast<T, BPS, DM_F32OUT>((T)zc.x, (T)zc.y, cons, c, v);
                // declined symbols go to the list for k_demap_fix (which rewrites their
                // plane entries): one atomic per wave, entries by lane rank
                const unsigned long long m = __ballot(dec);
                if (m) {
                    const int leader = __ffsll((long long)m) - 1;
                    unsigned base = 0;
                    if (me == leader) base = atomicAdd(dd.count, (unsigned)__popcll(m));
                    base = __shfl(base, leader);
                    if (dec) {
                        const unsigned e = base + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                                           __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
                        if (e < dd.cap) dd.list[e] = make_int2((int)cw, (int)s);
                        else dd.ovf[tile] = 1;
                    }
                }
                if (!live || dec) continue;
            } else {
                if (!live) continue;
                demap_sym<T, BPS, DM_F32OUT>((T)zc.x, (T)zc.y, cons, c, v);
            }
#pragma unroll
            for (int b = 0; b < BPS; ++b) L[ln * LD + b * ns + sx] = (float)v[b];
        }
        float *base = planes + tile * tile_floats(N);
        __syncthreads();
        for (int t = threadIdx.x; t < WAVE * (k1 - k0) * 2; t += BLOCK) {
            const int lane = t & (WAVE - 1);
            const int q = __builtin_amdgcn_readfirstlane(t >> 6);   // (step, half): wave-uniform, so src[] is read by scalar loads
            const int k = k0 + q / 2, half = q & 1;
            const long cw = tile * WAVE + lane;
            const int nc = half ? 2 : 4;
            float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                if (cc >= nc) break;
                const int j = src[(long)(half ? 6 + cc : cc) * N + k];
                const int col = j >= 0 ? (j % BPS) * ns + (int)(j / BPS - s0) : 0;
                v[cc] = (j >= 0 && j < n_avail && cw < B) ? L[lane * LD + col] : 0.0f;
            }
            if (half == 0) reinterpret_cast<float4 *>(base)[(long)k * WAVE + lane] = make_float4(v[0], v[1], v[2], v[3]);
            else reinterpret_cast<float2 *>(base + (long)N * WAVE * 4)[(long)k * WAVE + lane] = make_float2(v[0], v[1]);
        }
        __syncthreads();   // L is rewritten by the next item: its reads done everywhere
    }
}

// The declined symbols of k_demap_planes (split tables): demap_sym's whole chain,
// each LLR into its plane entry (dst[j] = c * N + k for the component c of couple
// k that LLR j feeds, -1: none), then every symbol of an overflowed tile.
template <typename T, int BPS>
__device__ __forceinline__ void dm_fix_symbol(long cw, long s, int N, int S, const float *syms, const T *cons,
                                              const DemapCfg &c, const int *dst, long n_avail, float *planes) {
    const float2 z = *reinterpret_cast<const float2 *>(syms + 2 * (cw * S + s));
    double v[BPS];
    demap_sym<T, BPS, DM_F32OUT>((T)z.x, (T)z.y, cons, c, v);
    float *base = planes + (cw / WAVE) * tile_floats(N);
    const int lane = (int)(cw & (WAVE - 1));
#pragma unroll
    for (int b = 0; b < BPS; ++b) {
        const long j = s * BPS + b;
        if (j >= n_avail) break;
        const int d = dst[j];
        if (d < 0) continue;
        const int cc = d / N, k = d - cc * N;
        if (cc < 4) base[((long)k * WAVE + lane) * 4 + cc] = (float)v[b];
        else base[(long)N * WAVE * 4 + ((long)k * WAVE + lane) * 2 + (cc - 6)] = (float)v[b];
    }
}
template <typename T, int BPS>
__global__ __launch_bounds__(BLOCK) void k_demap_fix(int B, int N, int S, const float *syms, const T *cons_g,
                                                    DemapCfg c, const int *__restrict__ dst, long n_avail,
                                                    float *planes, DemapDecl dd, long n_tiles) {
    __shared__ T cons[DM_TAB];
    load_table<T, BPS>(cons, cons_g, c);
    __syncthreads();
    const unsigned n = min(*dd.count, dd.cap);
    for (unsigned i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) {
        const int2 e = dd.list[i];
        if (dd.ovf[e.x / WAVE]) continue;   // redone below
        dm_fix_symbol<T, BPS>(e.x, e.y, N, S, syms, cons, c, dst, n_avail, planes);
    }
    for (long t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        if (!dd.ovf[t]) continue;
        for (long i = threadIdx.x; i < (long)WAVE * S; i += BLOCK) {
            const long cw = t * WAVE + i / S;
            if (cw < B) dm_fix_symbol<T, BPS>(cw, i % S, N, S, syms, cons, c, dst, n_avail, planes);
        }
    }
}

// ---- fused demap + decode ------------------------------------------------------------
// Each persistent decoder wave demaps its next 64-codeword tile itself (the same
// operations as k_demap_planes, so the planes are bit-identical) into a plane
// buffer of its own, then decodes it.  The demap is VALU-bound and the decoder
// HBM-bound, so inside one launch the demap's arithmetic runs while the other
// waves stream the decoder's planes (a separate k_demap_planes launch serialises
// them), and the plane buffer is sized per resident wave, not per codeword.
constexpr int DF_KC = 8;                   // couples per LDS chunk
constexpr int DF_LD = DF_KC * 6 + 1;       // odd row stride

struct FusedDemapArgs {
    const float *syms;                     // [B][S] complex64
    int S;
    long n_avail;                          // LLRs the symbols provide (<= the de-puncture walk)
    const int *src, *off;                  // de-puncture map (tdec_create)
    float *planes_w;                       // [n_waves][2] x tile_floats(N): the wave's current and next tile
    DemapCfg c;
    const void *cons_g;                    // device table (T)
};

template <typename T, int BPS> struct DemapPro {
    FusedDemapArgs a;                       // by value: SGPRs, no address of a kernel argument
    int B;
    const T *cons;                          // LDS copy
    float *L;                               // this wave's LDS chunk [64][DF_LD]
    __device__ __forceinline__ const float *tile_planes(int /*tile*/, int wave, int N, int buf) const {
        return a.planes_w + (2L * wave + buf) * tile_floats(N);
    }
    // chunks [piece/npieces, (piece+1)/npieces) of the tile's DF_KC-couple chunks
    __device__ __forceinline__ void fill(int tile, int wave, int N, int buf, int piece, int npieces) const {
        const int lane = threadIdx.x & (WAVE - 1);
        float *pl = a.planes_w + (2L * wave + buf) * tile_floats(N);
        float4 *X = reinterpret_cast<float4 *>(pl);
        float2 *Z = reinterpret_cast<float2 *>(pl + (long)N * WAVE * 4);
        const int S = a.S;
        const int nch = (N + DF_KC - 1) / DF_KC;
        const int c0 = piece * nch / npieces, c1 = (piece + 1) * nch / npieces;
        for (int ch = c0; ch < c1; ++ch) {
            const int k0 = ch * DF_KC, k1 = min(N, k0 + DF_KC);
            const long j0 = a.off[k0], j1 = a.off[k1];
            const long s0 = j0 / BPS, s1 = (j1 + BPS - 1) / BPS;   // symbols covering [j0, j1)
            const int ns = (int)(s1 - s0);
            for (int t = lane; t < WAVE * ns; t += WAVE) {
                const int l = t / ns, si = t - l * ns;              // consecutive lanes: consecutive symbols
                const long cw = (long)tile * WAVE + l;
                const long sy = s0 + si;
                if (cw >= B || sy >= S) continue;
                const float2 z = *reinterpret_cast<const float2 *>(a.syms + 2 * (cw * S + sy));
                double v[BPS];
                demap_sym<T, BPS, DM_F32OUT>((T)z.x, (T)z.y, cons, a.c, v);
#pragma unroll
                for (int b = 0; b < BPS; ++b) {
                    const long j = sy * BPS + b;
                    if (j >= j0 && j < j1) L[l * DF_LD + (int)(j - j0)] = (float)v[b];
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const long cw = (long)tile * WAVE + lane;
            for (int k = k0; k < k1; ++k) {
                float v[6];
#pragma unroll
                for (int cc = 0; cc < 6; ++cc) {
                    const int j = a.src[(long)(cc < 4 ? cc : cc + 2) * N + k];
                    v[cc] = (j >= 0 && j < a.n_avail && cw < B) ? L[lane * DF_LD + (int)(j - j0)] : 0.0f;
                }
                X[(long)k * WAVE + lane] = make_float4(v[0], v[1], v[2], v[3]);
                Z[(long)k * WAVE + lane] = make_float2(v[4], v[5]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    // the decoder reads the filled planes back through the CU's vector L1, which
    // may hold lines of the buffer's previous tile: publish the stores, invalidate L1
    __device__ __forceinline__ void publish() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
};

template <int ALGO, bool RAG, typename T, int BPS>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(DEC_WPE))) void
k_turbo_decode_syms(DecodeArgs p, const int *__restrict__ perm, const int *__restrict__ inv,
                    const int *__restrict__ used, FusedDemapArgs fa) {
    __shared__ uint32_t epi[WAVES_PER_BLOCK * 2 * WAVE];
    __shared__ T cons[DM_TAB];
    __shared__ float L[WAVES_PER_BLOCK * WAVE * DF_LD];
    load_table<T, BPS>(cons, reinterpret_cast<const T *>(fa.cons_g), fa.c);
    __syncthreads();
    DemapPro<T, BPS> pro{fa, p.B, cons, L + (threadIdx.x >> 6) * WAVE * DF_LD};
    turbo_decode_tiles<ALGO, RAG>(p, perm, inv, used, nullptr, nullptr, epi, pro);
}

// ---- encoder (workload generation; encode, :404-462) ------------------------------
struct EncodeArgs {
    int B, N, period;
    long n_out;
    unsigned char punct[16];
    int circ[16];
    const int *perm;
    const uint8_t *bits;
    uint8_t *coded;
};

__device__ __forceinline__ int next_rt(int s, int inp) {
    const int dk = ((inp >> 1) & 1) ^ (inp & 1) ^ ((s >> 2) & 1) ^ ((s >> 3) & 1);
    return (((s >> 2) & 1) << 3) | (((s >> 1) & 1) << 2) | ((s & 1) << 1) | dk;
}

__global__ __launch_bounds__(BLOCK) void k_encode(EncodeArgs p) {
    const long cw = (long)blockIdx.x * BLOCK + threadIdx.x;
    if (cw >= p.B) return;
    const uint8_t *u = p.bits + cw * 2 * p.N;
    uint8_t *o = p.coded + cw * p.n_out;
    int s1 = 0, s2 = 0;
    for (int i = 0; i < p.N; ++i) {
        const int j = p.perm[i];
        s1 = next_rt(s1, (u[2 * i] << 1) | u[2 * i + 1]);
        s2 = next_rt(s2, (u[2 * j] << 1) | u[2 * j + 1]);
    }
    s1 = p.circ[s1];
    s2 = p.circ[s2];
    long q = 0;
    for (int i = 0; i < p.N; ++i) {
        const int j = p.perm[i], ph = i % p.period;
        const int i1 = (u[2 * i] << 1) | u[2 * i + 1], i2 = (u[2 * j] << 1) | u[2 * j + 1];
        const int dk1 = ((i1 >> 1) & 1) ^ (i1 & 1) ^ ((s1 >> 2) & 1) ^ ((s1 >> 3) & 1);
        const int dk2 = ((i2 >> 1) & 1) ^ (i2 & 1) ^ ((s2 >> 2) & 1) ^ ((s2 >> 3) & 1);
        o[q++] = u[2 * i];
        o[q++] = u[2 * i + 1];
        if (p.punct[0 * 4 + ph]) o[q++] = dk1 ^ (s1 & 1) ^ ((s1 >> 1) & 1) ^ ((s1 >> 3) & 1);
        if (p.punct[1 * 4 + ph]) o[q++] = dk1 ^ ((s1 >> 1) & 1) ^ ((s1 >> 2) & 1) ^ ((s1 >> 3) & 1);
        if (p.punct[2 * 4 + ph]) o[q++] = dk2 ^ (s2 & 1) ^ ((s2 >> 1) & 1) ^ ((s2 >> 3) & 1);
        if (p.punct[3 * 4 + ph]) o[q++] = dk2 ^ ((s2 >> 1) & 1) ^ ((s2 >> 2) & 1) ^ ((s2 >> 3) & 1);
        s1 = next_rt(s1, i1);
        s2 = next_rt(s2, i2);
    }
}

}  // namespace tdec
