// tdec_lowlat.hip -- low-latency turbo decode for small batches (max-log):
// ONE STATE PER LANE.
//
// The throughput decoder (k_turbo_decode) runs one codeword per lane, so a
// single codeword is one lane of one wave walking every trellis step of all 16
// SISOs serially: a decode() call (test.py:81, one frame per call) takes one
// wave's full instruction stream.  Here a 16-lane group (one DPP row) holds the
// 16 state metrics of one codeword, 4 codewords per wave: each lane does one
// state's share of a step, predecessor / successor metrics come from the other
// lanes (ds_bpermute), state 0 is broadcast for the normalisation and the
// extrinsic's maxima over the states are row reductions (DPP row rotations).
// The same f32 / f64 operations as bcjr_max_log_map (dvb_rcs2_turbo.py:116-281)
// and the per-lane kernel, so the result is bit-exact (maxima are exact and
// order-free; tests/test_gpu_lowlat.py).
//
// Passes per SISO: F1 (alpha1 from 0, every alpha stored), F2 (from alpha1[N]
// until it equals the stored alpha1, per codeword), B1 (beta1 from 0 with the
// provisional extrinsic from alpha2 and beta1, every beta1 stored), B2 (from
// beta1[0], recomputing the extrinsic until beta2 equals beta1).  Per codeword
// the workspace is a few hundred KB (alpha / beta stores, extrinsic planes), so
// a small batch lives in L2; loads run 8 steps ahead of their use.
//
// No cross-lane memory traffic: every lane of a group stores the group's
// (identical) extrinsic values and reads back its own stores, each lane its own
// state's alpha / beta slot.
namespace tdec {

struct LLArgs {
    int B, N, iters;
    const float *planes;   // tile layout of k_depuncture / k_demap_planes
    double2 *ws;           // per codeword [3][N]: P1, Le2, Le1
    float *st;             // per codeword [2][N + 1][16]: alpha store, beta store
    int32_t *bits;         // [B][2N]
    double *lfinal;        // [B][2N] or null
};
__host__ __device__ constexpr long ll_ws_elems(int N) { return 3L * N; }
__host__ __device__ constexpr long ll_st_elems(int N) { return 2L * (N + 1) * 16; }

// max over the 16 lanes of a DPP row (rotations: every lane ends with the maximum)
__device__ __forceinline__ float row_max16(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false)));   // row_ror:8
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false)));   // row_ror:4
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xF, 0xF, false)));   // row_ror:2
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xF, 0xF, false)));   // row_ror:1
    return v;
}
// true when all 16 lanes of the calling lane's group have c set (group-uniform)
__device__ __forceinline__ bool group_all(bool c, int base) {
    const unsigned long long m = __ballot(c);
    return ((m >> base) & 0xFFFFull) == 0xFFFFull;
}

// The raw inputs of one step, identical in the 16 lanes of a group.
struct LLRaw {
    float4 v;    // {Lc_A, Lc_B, W, Y}   (decoder 2: {-, -, W2, Y2})
    double2 l;   // decoder 1: La = Le2[inv[k]]; decoder 2: P1[perm[k]] = f64(Lc) + La
};

struct LLIn1 {   // decoder 1: natural order, a-priori Le2[inv_perm[k]] (0 in the first iteration)
    const float4 *X;
    const double2 *Le2;
    const int *inv;
    int cwl;     // lane of the codeword inside its tile
    bool first;
    __device__ __forceinline__ LLRaw load(int k) const {
        LLRaw r;
        r.v = X[(long)k * WAVE + cwl];
        r.l = first ? make_double2(0.0, 0.0) : Le2[inv[k]];
        return r;
    }
    __device__ __forceinline__ void gamma(const LLRaw &r, float (&g)[8], double &iA, double &iB) const {
        make_gamma(r.v.x, r.v.y, r.l.x, r.l.y, r.v.z, r.v.w, g, iA, iB);
    }
};
struct LLIn2 {   // decoder 2: {W2, Y2} and the pre-summed P1[perm[k]] (:511-516)
    const float2 *Z;
    const double2 *P1;
    const int *perm;
    int cwl;
    __device__ __forceinline__ LLRaw load(int k) const {
        LLRaw r;
        const float2 z = Z[(long)k * WAVE + cwl];
        r.v = make_float4(0.0f, 0.0f, z.x, z.y);
        r.l = P1[perm[k]];
        return r;
    }
    __device__ __forceinline__ void gamma(const LLRaw &r, float (&g)[8], double &iA, double &iB) const {
        iA = r.l.x;
        iB = r.l.y;
        gamma_from_sums(iA, iB, r.v.z, r.v.w, g);
    }
};
struct LLOut1 {  // P1 = f64(Lc) + Le1 for decoder 2, Le1 itself in the last iteration
    double2 *P1, *Le1;
    bool live;
    __device__ __forceinline__ void store(int k, double a, double b, float lcA, float lcB) const {
        if (!live) return;
        P1[k] = make_double2((double)lcA + a, (double)lcB + b);
        if (Le1) Le1[k] = make_double2(a, b);
    }
};
struct LLOut2 {
    double2 *Le2;
    bool live;
    __device__ __forceinline__ void store(int k, double a, double b, float, float) const {
        if (live) Le2[k] = make_double2(a, b);
    }
};

__device__ __forceinline__ void ll_pm(const float (&g)[8], float (&pm)[8]) {
    float p2[2][4];
    pair_max(g, p2);
#pragma unroll
    for (int i = 0; i < 8; ++i) pm[i] = p2[i >> 2][i & 3];
}

// extrinsic of one position (:232-281) from this lane's alpha and the group's beta
__device__ __forceinline__ void ll_extrinsic(float a, float b, const float (&g)[8], const SplLane &L, double iA,
                                             double iB, double sf, double &leA, double &leB) {
    const float bx = __shfl(b, L.base + L.nxt[0]), by = __shfl(b, L.base + L.nxt[1]);   // next(s,3) = next(s,0) etc.
    float app[4];
#pragma unroll
    for (int inp = 0; inp < 4; ++inp) {
        const float gv = sel8(g, L.gi[inp]);
        const float t = (a + (L.gn[inp] ? -gv : gv)) + ((inp == 0 || inp == 3) ? bx : by);
        app[inp] = row_max16(fmaxf(NEG, t));
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

constexpr int LL_D = 8;   // loads issued this many steps ahead of their use

// One SISO (:116-281) of the group's codeword.  ast / bst: this codeword's
// alpha / beta stores [N + 1][16] (this lane: element s of each row).
template <class In, class Out>
__device__ void ll_siso(const In &in, const Out &out, int N, float *ast, float *bst, const SplLane &L, double sf) {
    const int s = L.s;
    LLRaw r[LL_D];
    float g[8], pm[8];
    double iA, iB;
    // F1: alpha1 from 0, every step stored
    float a = 0.0f;
#pragma unroll
    for (int j = 0; j < LL_D; ++j) r[j] = in.load(min(j, N - 1));
    for (int k0 = 0; k0 < N; k0 += LL_D) {
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            const int k = k0 + j;
            if (k >= N) break;   // wave-uniform
            in.gamma(r[j], g, iA, iB);
            r[j] = in.load(min(k + LL_D, N - 1));
            ll_pm(g, pm);
            ast[k * 16 + s] = a;
            a = spl_alpha(a, pm, L);
        }
    }
    // F2 from alpha1[N] until alpha2 == alpha1 (per codeword: all 16 lanes of the group)
    bool merged = false;
#pragma unroll
    for (int j = 0; j < LL_D; ++j) r[j] = in.load(min(j, N - 1));
    for (int k0 = 0; k0 < N && !__all(merged); k0 += LL_D) {
        float c[LL_D];
#pragma unroll
        for (int j = 0; j < LL_D; ++j) c[j] = ast[min(k0 + j, N - 1) * 16 + s];
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            const int k = k0 + j;
            if (k >= N) break;
            if (!merged) merged = group_all(a == c[j], L.base);
            in.gamma(r[j], g, iA, iB);
            r[j] = in.load(min(k + LL_D, N - 1));
            if (!merged) {
                ll_pm(g, pm);
                ast[k * 16 + s] = a;
                a = spl_alpha(a, pm, L);
            }
        }
    }
    // B1: beta1 from 0 with the provisional extrinsic (alpha2, beta1); beta1[k+1] stored
    float b = 0.0f;
#pragma unroll
    for (int j = 0; j < LL_D; ++j) r[j] = in.load(max(N - 1 - j, 0));
    for (int k0 = N - 1; k0 >= 0; k0 -= LL_D) {
        float av[LL_D];
#pragma unroll
        for (int j = 0; j < LL_D; ++j) av[j] = ast[max(k0 - j, 0) * 16 + s];
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            const int k = k0 - j;
            if (k < 0) break;
            in.gamma(r[j], g, iA, iB);
            const float lcA = r[j].v.x, lcB = r[j].v.y;
            r[j] = in.load(max(k - LL_D, 0));
            double leA, leB;
            ll_extrinsic(av[j], b, g, L, iA, iB, sf, leA, leB);
            out.store(k, leA, leB, lcA, lcB);
            bst[(k + 1) * 16 + s] = b;
            ll_pm(g, pm);
            b = spl_beta(b, pm, L);
        }
    }
    // B2 from beta1[0] until beta2 == beta1: below that the provisional values are exact
    merged = false;
#pragma unroll
    for (int j = 0; j < LL_D; ++j) r[j] = in.load(max(N - 1 - j, 0));
    for (int k0 = N - 1; k0 >= 0 && !__all(merged); k0 -= LL_D) {
        float av[LL_D], c[LL_D];
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            av[j] = ast[max(k0 - j, 0) * 16 + s];
            c[j] = bst[(max(k0 - j, 0) + 1) * 16 + s];
        }
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            const int k = k0 - j;
            if (k < 0) break;
            if (!merged) merged = group_all(b == c[j], L.base);
            in.gamma(r[j], g, iA, iB);
            const float lcA = r[j].v.x, lcB = r[j].v.y;
            r[j] = in.load(max(k - LL_D, 0));
            if (!merged) {
                double leA, leB;
                ll_extrinsic(av[j], b, g, L, iA, iB, sf, leA, leB);
                out.store(k, leA, leB, lcA, lcB);
                ll_pm(g, pm);
                b = spl_beta(b, pm, L);
            }
        }
    }
}

// DVBRCS2_Turbo.decode (:464-537) for 4 codewords per wave, one wave per block.
__global__ __launch_bounds__(WAVE) void k_turbo_decode_lowlat(LLArgs p, const int *__restrict__ perm,
                                                              const int *__restrict__ inv) {
    const int lane = threadIdx.x;
    const long cw0 = (long)blockIdx.x * 4 + (lane >> 4);
    const bool live = cw0 < p.B;
    const long cw = live ? cw0 : p.B - 1;    // idle groups shadow the last codeword and store nothing
    const SplLane L = spl_lane(lane);
    const int N = p.N;
    const long tile = cw / WAVE;
    const int cwl = (int)(cw % WAVE);
    const float *base = p.planes + tile * tile_floats(N);
    const float4 *X = reinterpret_cast<const float4 *>(base);
    const float2 *Z = reinterpret_cast<const float2 *>(base + (long)N * WAVE * 4);
    // idle groups get their own workspace slot (the one after the batch), never read back
    const long slot = live ? cw : p.B + (lane >> 4);
    double2 *P1 = p.ws + slot * ll_ws_elems(N), *Le2 = P1 + N, *Le1 = Le2 + N;
    float *ast = p.st + slot * ll_st_elems(N), *bst = ast + (N + 1) * 16;
    for (int it = 0; it < p.iters; ++it) {
        const double sf = it < p.iters - 1 ? 0.7 : 1.0;   // :496
        const bool last = it == p.iters - 1;
        ll_siso(LLIn1{X, Le2, inv, cwl, it == 0}, LLOut1{P1, last ? Le1 : nullptr, live}, N, ast, bst, L, sf);
        ll_siso(LLIn2{Z, P1, perm, cwl}, LLOut2{Le2, live}, N, ast, bst, L, sf);
    }
    // hard decision (:526-537): L = (Lc + La) + Le1, La = Le2[inv_perm]; lane s takes k = s, s + 16, ...
    if (!live) return;
    for (int k = L.s; k < N; k += 16) {
        const float4 x = X[(long)k * WAVE + cwl];
        const double2 la = Le2[inv[k]], le = Le1[k];
        const double fa = ((double)x.x + la.x) + le.x;
        const double fb = ((double)x.y + la.y) + le.y;
        *reinterpret_cast<int2 *>(p.bits + cw * 2 * N + 2 * k) = make_int2(fa < 0.0 ? 1 : 0, fb < 0.0 ? 1 : 0);
        if (p.lfinal) *reinterpret_cast<double2 *>(p.lfinal + cw * 2 * N + 2 * k) = make_double2(fa, fb);
    }
}

}  // namespace tdec
