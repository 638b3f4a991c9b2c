// tdec_spl.hip -- A/B prototype of the north star's mapping for the SISO
// (DESIGN.md §3): ONE STATE PER LANE.  16 lanes hold the 16
// state metrics of one codeword (4 codewords per wave); every trellis step
// exchanges predecessor / successor metrics between lanes (ds_bpermute via
// __shfl) and broadcasts state 0 for the normalisation; the extrinsic's
// maxima over the 16 states are butterfly reductions across the 16 lanes.
// Same f32 / f64 operations as bcjr_max_log_map (:116-281) and the per-lane
// kernel, so the result is bit-exact (maxima are exact and order-free).
//
// It exists to be timed against k_siso_batch (the per-lane mapping, one
// codeword per lane) on the same inputs: tdec_siso_batch runs it when
// TDEC_SISO_SPL=1.  Not used by the product.
#include <hip/hip_runtime.h>

namespace tdec {

constexpr int SPL_W = 4;                 // alpha checkpoint interval
constexpr int SPL_G = 16;                // lanes per codeword

struct SplRow {
    const float *A, *B, *W, *Y;
    const double *LaA, *LaB;
};

// pm index of branch pair (p, inp): pm[t][wy] flattened t*4 + wy
__device__ __forceinline__ int spl_pm_idx(int p, int inp) {
    const int t = ((((inp >> 1) & 1) ^ (inp & 1) ^ ((p >> 2) & 1) ^ ((p >> 3) & 1)) ^ ((p >> 2) & 1) ^ ((p >> 3) & 1));
    const int dk = ((inp >> 1) & 1) ^ (inp & 1) ^ ((p >> 2) & 1) ^ ((p >> 3) & 1);
    const int w = dk ^ (p & 1) ^ ((p >> 1) & 1) ^ ((p >> 3) & 1), y = dk ^ ((p >> 1) & 1) ^ ((p >> 2) & 1) ^ ((p >> 3) & 1);
    return t * 4 + w * 2 + y;
}
// gamma index of branch (s, inp) into g8 with sign: g(bA=0, ...) = g[bB*4+bW*2+bY]; bA=1 -> -g[~bits]
__device__ __forceinline__ int spl_g_idx(int s, int inp, bool &neg) {
    const int dk = ((inp >> 1) & 1) ^ (inp & 1) ^ ((s >> 2) & 1) ^ ((s >> 3) & 1);
    const int bA = (inp >> 1) & 1, bB = inp & 1;
    const int bW = dk ^ (s & 1) ^ ((s >> 1) & 1) ^ ((s >> 3) & 1), bY = dk ^ ((s >> 1) & 1) ^ ((s >> 2) & 1) ^ ((s >> 3) & 1);
    neg = bA == 1;
    return bA == 0 ? bB * 4 + bW * 2 + bY : (bB ^ 1) * 4 + (bW ^ 1) * 2 + (bY ^ 1);
}
__device__ __forceinline__ float sel8(const float (&v)[8], int i) {
    const float a = (i & 1) ? v[1] : v[0], b = (i & 1) ? v[3] : v[2], c = (i & 1) ? v[5] : v[4], d = (i & 1) ? v[7] : v[6];
    const float e = (i & 2) ? b : a, f = (i & 2) ? d : c;
    return (i & 4) ? f : e;
}

struct SplLane {            // per-lane constants of the state this lane holds
    int s, base;            // state, first lane of the codeword's group
    int srcA, srcB;         // lanes of the two predecessors (alpha)
    int pmA, pmB;           // their branch-pair indices into pm
    int sucA, sucB;         // lanes of the two successors (beta): next(s, ie) and its pair
    int pmS0, pmS1;         // branch pairs of s towards sucA / sucB
    int gi[4];              // gamma index of (s, inp)
    bool gn[4];
    int nxt[4];             // next(s, inp) - base
};

__device__ __forceinline__ SplLane spl_lane(int lane) {
    SplLane L;
    L.s = lane & (SPL_G - 1);
    L.base = lane & ~(SPL_G - 1);
    const int p0 = t_prev_s(L.s, 0), p1 = t_prev_s(L.s, 2);
    L.srcA = L.base + p0;
    L.srcB = L.base + p1;
    L.pmA = spl_pm_idx(p0, t_prev_i(L.s, 0));
    L.pmB = spl_pm_idx(p1, t_prev_i(L.s, 2));
    const int ie = (t_next(L.s, 0) & 1) ? 1 : 0;           // input to the even successor
    const int ne = t_next(L.s, ie);
    L.sucA = L.base + ne;
    L.sucB = L.base + ne + 1;
    L.pmS0 = spl_pm_idx(L.s, ie);
    L.pmS1 = spl_pm_idx(L.s, ie ^ 1);
    for (int i = 0; i < 4; ++i) {
        L.gi[i] = spl_g_idx(L.s, i, L.gn[i]);
        L.nxt[i] = t_next(L.s, i);
    }
    return L;
}

__device__ __forceinline__ void spl_gamma(const SplRow &r, int k, float (&g)[8], float (&pm)[8], double &iA, double &iB) {
    make_gamma(r.A[k], r.B[k], r.LaA[k], r.LaB[k], r.W[k], r.Y[k], g, iA, iB);
    float p2[2][4];
    pair_max(g, p2);
#pragma unroll
    for (int i = 0; i < 8; ++i) pm[i] = p2[i >> 2][i & 3];
}

__device__ __forceinline__ float spl_alpha(float a, const float (&pm)[8], const SplLane &L) {
    const float x = __shfl(a, L.srcA) + sel8(pm, L.pmA);
    const float y = __shfl(a, L.srcB) + sel8(pm, L.pmB);
    const float n = fmaxf(fmaxf(NEG, x), y);
    return n - __shfl(n, L.base);
}
__device__ __forceinline__ float spl_beta(float b, const float (&pm)[8], const SplLane &L) {
    const float x = __shfl(b, L.sucA) + sel8(pm, L.pmS0);
    const float y = __shfl(b, L.sucB) + sel8(pm, L.pmS1);
    const float n = fmaxf(fmaxf(NEG, x), y);
    return n - __shfl(n, L.base);
}

__device__ __forceinline__ float spl_max16(float v) {
#pragma unroll
    for (int o = 1; o < SPL_G; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// Extrinsic of one position: app[inp] = max_s (alpha[s] + gamma(s, inp)) + beta[next(s, inp)]
__device__ __forceinline__ void spl_extrinsic(float a, float b1, const float (&g)[8], const SplLane &L, double iA,
                                              double iB, double sf, double &leA, double &leB) {
    float app[4];
#pragma unroll
    for (int inp = 0; inp < 4; ++inp) {
        const float gv = sel8(g, L.gi[inp]);
        const float t = (a + (L.gn[inp] ? -gv : gv)) + __shfl(b1, L.base + L.nxt[inp]);
        app[inp] = spl_max16(fmaxf(NEG, t));
    }
    const float pA0 = app[0] > app[1] ? app[0] : app[1], pA1 = app[2] > app[3] ? app[2] : app[3];
    const float pB0 = app[0] > app[2] ? app[0] : app[2], pB1 = app[1] > app[3] ? app[1] : app[3];
    double x = ((double)(pA0 - pA1) - iA) * sf, y = ((double)(pB0 - pB1) - iB) * sf;
    x = x > 300.0 ? 300.0 : x;
    x = x < -300.0 ? -300.0 : x;
    y = y > 300.0 ? 300.0 : y;
    y = y < -300.0 ? -300.0 : y;
    leA = x;
    leB = y;
}

struct SplArgs {
    int B, N;
    const float *LcA, *LcB, *LcW, *LcY;
    const double *LaA, *LaB;
    double sf;
    double *LeA, *LeB;
    float *ck;            // [grid waves][ceil(N/W) + RING][64] floats
    long ck_stride;       // floats per wave
};

__global__ __launch_bounds__(256) void k_siso_spl(SplArgs p) {
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long cw = wave * 4 + (lane >> 4);
    const bool live = cw < p.B;
    if (__all(!live)) return;
    const long row = (live ? cw : p.B - 1) * p.N;
    const SplRow r{p.LcA + row, p.LcB + row, p.LcW + row, p.LcY + row, p.LaA + row, p.LaB + row};
    const SplLane L = spl_lane(lane);
    const int N = p.N, nw = (N + SPL_W - 1) / SPL_W;
    float *ck = p.ck + wave * p.ck_stride;
    float *ring = ck + (long)nw * 64;
    float g[8], pm[8];
    double iA, iB;
    // F1: alpha1 from 0, checkpoint every SPL_W steps
    float a = 0.0f;
    for (int k = 0; k < N; ++k) {
        if (k % SPL_W == 0) ck[(k / SPL_W) * 64 + lane] = a;
        spl_gamma(r, k, g, pm, iA, iB);
        a = spl_alpha(a, pm, L);
    }
    // F2 from alpha1[N] until the whole wave has merged at a checkpoint
    for (int k = 0; k < N; ++k) {
        if (k % SPL_W == 0) {
            if (__all(a == ck[(k / SPL_W) * 64 + lane])) break;
            ck[(k / SPL_W) * 64 + lane] = a;
        }
        spl_gamma(r, k, g, pm, iA, iB);
        a = spl_alpha(a, pm, L);
    }
    // B1 (provisional extrinsic) and B2 (until merged with beta1 at a kept window start)
    float b = 0.0f;
    const int top = ((N - 1) / SPL_W) * SPL_W;
    for (int pass = 0; pass < 2; ++pass) {
        for (int k0 = top; k0 >= 0; k0 -= SPL_W) {
            const int rw = (top - k0) / SPL_W;
            const bool keep = rw % 4 == 0 && rw < RING * 4;
            if (keep) {
                if (pass == 0) ring[(rw / 4) * 64 + lane] = b;
                else if (__all(b == ring[(rw / 4) * 64 + lane])) break;
            }
            const int len = min(SPL_W, N - k0);     // wave-uniform
            float aw[SPL_W], gw[SPL_W][8], pw[SPL_W][8];
            double iAw[SPL_W], iBw[SPL_W];
#pragma unroll
            for (int j = 0; j < SPL_W; ++j)
                if (j < len) spl_gamma(r, k0 + j, gw[j], pw[j], iAw[j], iBw[j]);
            aw[0] = ck[(k0 / SPL_W) * 64 + lane];
#pragma unroll
            for (int j = 1; j < SPL_W; ++j)
                if (j < len) aw[j] = spl_alpha(aw[j - 1], pw[j - 1], L);
#pragma unroll
            for (int j = SPL_W - 1; j >= 0; --j) {
                if (j >= len) continue;
                double leA, leB;
                spl_extrinsic(aw[j], b, gw[j], L, iAw[j], iBw[j], p.sf, leA, leB);
                if (live && L.s == 0) {
                    p.LeA[row + k0 + j] = leA;
                    p.LeB[row + k0 + j] = leB;
                }
                b = spl_beta(b, pw[j], L);
            }
        }
    }
}

}  // namespace tdec
