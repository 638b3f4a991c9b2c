// tdec_lowlat.hip -- low-latency turbo decode for small batches (max-log):
// ONE CODEWORD PER WAVE, ONE STATE PER LANE.
//
// The throughput decoder (k_turbo_decode) runs one codeword per lane, so a
// single codeword is one lane of one wave walking every trellis step of all 16
// SISOs serially: a decode() call (test.py:81, one frame per call) takes one
// wave's whole instruction stream.  Here a wave works on one codeword in four
// 16-lane groups (DPP rows), each lane one trellis state:
//   * recursions: group 0 runs alpha forward and group 1 runs beta backward AT
//     THE SAME TIME -- the two recursions do not depend on each other, and with
//     per-lane source lanes and branch-pair indices both are the same
//     instruction sequence (two ds_bpermute reads of the neighbours, add, max,
//     a third for the state-0 normalisation).  Pass 1 (F1 | B1) runs from 0
//     over the whole block storing every vector; pass 2 (F2 | B2) starts from
//     alpha1[N] / beta1[0] and overwrites the stored vectors until they equal
//     the stored pass-1 ones (per group; from there on they are identical);
//   * extrinsic: with every alpha2[k] and beta2[k+1] stored, the positions are
//     independent, so the 4 groups take 4 positions at a time: each lane forms
//     its state's 4 branch terms, the row maxima are DPP row rotations.
// The same f32 / f64 operations as bcjr_max_log_map (dvb_rcs2_turbo.py:116-281)
// and the per-lane kernel, so the result is bit-exact (maxima are exact and
// order-free; tests/test_gpu_lowlat.py).  Per codeword the workspace (alpha /
// beta stores, extrinsic planes) is ~130 KB, L2-resident for small batches;
// loads run 8 steps ahead of their use.  Lanes exchange stored vectors and
// extrinsics through memory, so a workgroup-scope fence separates the phases.
namespace tdec {

struct LLArgs {
    int B, N, iters;
    const float *planes;   // tile layout of k_depuncture / k_demap_planes
    double2 *ws;           // per codeword [3][N]: P1, Le2, Le1
    float *st;             // per codeword [2][N + 1][16]: alpha store, beta store
    int32_t *bits;         // [B][2N]
    double *lfinal;        // [B][2N] or null
    const int *ulist;      // [n_used]: the positions in perm's image, ascending
    int n_used;
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
// four row maxima, their rotation rounds interleaved (each DPP move reads a value
// written three instructions earlier: no hazard wait states)
template <int CTL> __device__ __forceinline__ void row_round4(float (&v)[4]) {
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v[i]), CTL, 0xF, 0xF, false));
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = fmaxf(v[i], o[i]);
}
__device__ __forceinline__ void row_max16x4(float (&v)[4]) {
    row_round4<0x128>(v);   // row_ror:8
    row_round4<0x124>(v);   // row_ror:4
    row_round4<0x122>(v);   // row_ror:2
    row_round4<0x121>(v);   // row_ror:1
}
// true when all 16 lanes of the calling lane's group have c set (group-uniform)
__device__ __forceinline__ bool group_all(bool c, int base) {
    const unsigned long long m = __ballot(c);
    return ((m >> base) & 0xFFFFull) == 0xFFFFull;
}
// stores of this wave visible to its later loads from any lane (the block is one wave)
__device__ __forceinline__ void ll_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// The raw inputs of one step.
struct LLRaw {
    float4 v;    // {Lc_A, Lc_B, W, Y}   (decoder 2: {-, -, W2, Y2})
    double2 l;   // decoder 1: La = Le2[inv[k]]; decoder 2: P1[perm[k]] = f64(Lc) + La
};

// The interleaver tables are staged in LDS at the kernel's start: the alpha and
// beta groups load different positions at the same instruction, so the index of
// a gather is a per-lane load, and as a vector load its s_waitcnt vmcnt(0) also
// waited for the 8-step-ahead input prefetches (every step paid the full memory
// latency); an LDS read only waits for LDS operations.
typedef __attribute__((address_space(3))) int lds_int;
struct LLIn1 {   // decoder 1: natural order, a-priori Le2[inv_perm[k]] (Le2 zeroed before the first iteration)
    const float4 *X;
    const double2 *Le2;
    const lds_int *inv;
    int cwl;     // lane of the codeword inside its tile
    __device__ __forceinline__ int ix(int k) const { return inv[k]; }
    __device__ __forceinline__ LLRaw load_ix(int k, int i) const {
        LLRaw r;
        r.v = X[(long)k * WAVE + cwl];
        r.l = Le2[i];
        return r;
    }
    __device__ __forceinline__ LLRaw load(int k) const { return load_ix(k, ix(k)); }
    __device__ __forceinline__ void gamma(const LLRaw &r, float (&g)[8], double &iA, double &iB) const {
        make_gamma(r.v.x, r.v.y, r.l.x, r.l.y, r.v.z, r.v.w, g, iA, iB);
    }
    __device__ __forceinline__ void sums(const LLRaw &r, double &iA, double &iB) const {
        iA = (double)r.v.x + r.l.x;   // make_gamma's f64 additions
        iB = (double)r.v.y + r.l.y;
    }
};
struct LLIn2 {   // decoder 2: {W2, Y2} and the pre-summed P1[perm[k]] (:511-516)
    const float2 *Z;
    const double2 *P1;
    const lds_int *perm;
    int cwl;
    __device__ __forceinline__ int ix(int k) const { return perm[k]; }
    __device__ __forceinline__ LLRaw load_ix(int k, int i) const {
        LLRaw r;
        const float2 z = Z[(long)k * WAVE + cwl];
        r.v = make_float4(0.0f, 0.0f, z.x, z.y);
        r.l = P1[i];
        return r;
    }
    __device__ __forceinline__ LLRaw load(int k) const { return load_ix(k, ix(k)); }
    __device__ __forceinline__ void gamma(const LLRaw &r, float (&g)[8], double &iA, double &iB) const {
        iA = r.l.x;
        iB = r.l.y;
        gamma_from_sums(iA, iB, r.v.z, r.v.w, g);
    }
    __device__ __forceinline__ void sums(const LLRaw &r, double &iA, double &iB) const {
        iA = r.l.x;
        iB = r.l.y;
    }
};
// The positions whose extrinsic is computed: i -> pos(i), i < count(N).  Before
// the last iteration decoder 1's output is read only as P1[perm[j]], so only the
// n_used positions in perm's image (355 of 752) are computed; in the last
// iteration every position.
struct LLOut1 {  // P1 = f64(Lc) + Le1 for decoder 2, Le1 itself in the last iteration
    double2 *P1, *Le1;
    const lds_int *ulist;   // LDS copy (a per-lane index, as the gathers')
    int n_used;
    __device__ __forceinline__ bool sparse() const { return !Le1; }
    __device__ __forceinline__ int count(int N) const { return sparse() ? n_used : N; }
    __device__ __forceinline__ int pos(int i) const { return sparse() ? ulist[i] : i; }
    __device__ __forceinline__ void store(int k, double a, double b, float lcA, float lcB) const {
        P1[k] = make_double2((double)lcA + a, (double)lcB + b);
        if (Le1) Le1[k] = make_double2(a, b);
    }
};
struct LLOut2 {
    double2 *Le2;
    __device__ __forceinline__ int count(int N) const { return N; }
    __device__ __forceinline__ int pos(int i) const { return i; }
    __device__ __forceinline__ void store(int k, double a, double b, float, float) const { Le2[k] = make_double2(a, b); }
};

// The branch metrics spread over the row instead of all 8 in every lane: lane j
// forms g[j & 7] only (gamma_from_sums's f64 operations for that
// element: the same bits), the pair maxima come from the quad partner by one DPP
// move (pm[t][wy] pairs g[t*4 + wy] with g[t*4 + 3 - wy], lanes j and j ^ 3), and
// each lane fetches the two pair maxima (extrinsic: the four metrics) it needs
// with permutes that do not wait on the recursion, instead of selecting them
// from 8 registers with cndmask chains.
__device__ __forceinline__ float gamma_lane(double inA, double inB, float w, float y, int i) {
    const double hA = inA * 0.5, hB = inB * 0.5, hW = (double)w * 0.5, hY = (double)y * 0.5;
    const double l1 = hA + (((i >> 2) & 1) ? -hB : hB);
    const double l2 = l1 + (((i >> 1) & 1) ? -hW : hW);
    return (float)(l2 + ((i & 1) ? -hY : hY));
}
// pair maximum pm[j & 7] of lane j's row: fmaxf(g[i], -g[i ^ 3]) as pair_max
__device__ __forceinline__ float pm_lane(float g) {
    const float o = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(g), 0x1B, 0xF, 0xF, false));   // quad_perm:[3,2,1,0]
    return fmaxf(g, -o);
}

// Per-lane constants: group 0 runs alpha (predecessors), group 1 beta (successors),
// in one instruction sequence: x = v[src0] + pm[i0], y = v[src1] + pm[i1].
struct LLRec {
    int src0, src1, i0, i1, base;
};
__device__ __forceinline__ LLRec ll_rec(const SplLane &L, bool beta) {
    return beta ? LLRec{L.sucA, L.sucB, L.pmS0, L.pmS1, L.base} : LLRec{L.srcA, L.srcB, L.pmA, L.pmB, L.base};
}
// state 0's value of the lane's 16-lane row: DPP row_newbcast:0 (gfx90a+), no LDS round trip
__device__ __forceinline__ float row_lane0(float n, int) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(n), 0x150, 0xF, 0xF, false));
}
template <class In> __device__ __forceinline__ void lane_pms(const In &in, const LLRaw &r, int s, const LLRec &R,
                                                            float &p0, float &p1) {
    double iA, iB;
    in.sums(r, iA, iB);
    const float pm = pm_lane(gamma_lane(iA, iB, r.v.z, r.v.w, s & 7));
    p0 = __shfl(pm, R.base + R.i0);
    p1 = __shfl(pm, R.base + R.i1);
}

constexpr int LL_D = 8;   // loads issued this many steps ahead of their use

// One SISO (:116-281) of the wave's codeword.  ast / bst: stores [N + 1][16]
// (lane s: element s); ast[k] = alpha2[k], bst[k] = beta2[k] on exit.
template <class In, class Out>
__device__ void ll_siso(const In &in, const Out &out, int N, float *ast, float *bst, const SplLane &L, int grp,
                        double sf) {
    const int s = L.s;
    if (grp < 2) {
        const bool beta = grp == 1;
        const LLRec R = ll_rec(L, beta);
        float *vst = beta ? bst : ast;
        // position of step k: alpha k, beta N - 1 - k; slot of the vector entering it:
        // alpha[k] (before the step), beta[pos + 1]
        auto pos = [&](int k) { return beta ? N - 1 - k : k; };
        auto slot = [&](int k) { return (beta ? N - k : k) * 16 + s; };
        LLRaw r[LL_D];
        float v = 0.0f;
        {
            // Software-pipelined: the next step's pair maxima (gamma's f64 chain and
            // two permutes) are formed while this step's neighbour permutes are in
            // flight, and the gather indices of the group after next are read from
            // LDS once per group, so no step waits on an index read.
            // Every step issues the same operations (no branch around a load or a
            // store: a merged group stores back the pass-1 value it compared
            // against), so the compiler's wait counts stay exact.
            // pair maxima two steps ahead: (c0, c1) for the next step, (n0, n1) for
            // the one after; a step waits only for its own neighbour permutes
            int ixn[LL_D];
            float c0, c1, n0, n1;
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                bool merged = false;
#pragma unroll
                for (int j = 0; j < LL_D; ++j) r[j] = in.load(pos(min(j, N - 1)));
#pragma unroll
                for (int j = 0; j < LL_D; ++j) ixn[j] = in.ix(pos(min(LL_D + j, N - 1)));
                lane_pms(in, r[0], s, R, c0, c1);
                lane_pms(in, r[1], s, R, n0, n1);
                // one trellis step (j: slot in the group, k: step)
                auto step = [&](int j, int k, const float (&c)[LL_D], const int (&ixc)[LL_D]) {
                    if (pass == 1 && !merged) merged = group_all(v == c[j], L.base);
                    const float p0 = c0, p1 = c1;
                    c0 = n0;
                    c1 = n1;
                    const float xa = __shfl(v, R.src0), ya = __shfl(v, R.src1);
                    // the permutes go out first; the branch metrics' f64 chain below
                    // then runs while they are in flight (the scheduler put it first)
                    __builtin_amdgcn_sched_barrier(0);
                    lane_pms(in, r[(j + 2) % LL_D], s, R, n0, n1);   // (past N: clamped rows, unused)
                    r[j] = in.load_ix(pos(min(k + LL_D, N - 1)), ixc[j]);
                    const float n = fmaxf(fmaxf(NEG, xa + p0), ya + p1);
                    const float vn = n - row_lane0(n, R.base);
                    const bool hold = pass == 1 && merged;
                    vst[slot(k)] = hold ? c[j] : v;
                    v = hold ? v : vn;
                };
                for (int k0 = 0; k0 < N; k0 += LL_D) {
                    if (pass == 1 && __all(merged || grp >= 2)) break;
                    float c[LL_D];
#pragma unroll
                    for (int j = 0; j < LL_D; ++j) c[j] = pass == 1 ? vst[slot(min(k0 + j, N - 1))] : 0.0f;
                    int ixc[LL_D];
#pragma unroll
                    for (int j = 0; j < LL_D; ++j) {
                        ixc[j] = ixn[j];
                        ixn[j] = in.ix(pos(min(k0 + 2 * LL_D + j, N - 1)));
                    }
                    if (k0 + LL_D <= N) {   // a whole group: straight-line code, no per-step branch
#pragma unroll
                        for (int j = 0; j < LL_D; ++j) step(j, k0 + j, c, ixc);
                    } else {
#pragma unroll
                        for (int j = 0; j < LL_D; ++j) {
                            if (k0 + j >= N) break;   // uniform
                            step(j, k0 + j, c, ixc);
                        }
                    }
                }
            }
        }
    }
    ll_sync();
    // extrinsic (:232-281) from the stored alpha2[k], beta2[k+1] at every position
    // anyone reads (out.pos(i), i < M): group q takes i = q, q + 4, ...
    const int nx0 = L.nxt[0], nx1 = L.nxt[1];   // next(s, 0) = next(s, 3), next(s, 1) = next(s, 2)
    const int M = out.count(N);
    for (int i0 = grp; i0 < M; i0 += 4 * LL_D) {
        LLRaw r[LL_D];
        float av[LL_D], bx[LL_D], by[LL_D];
        int kk[LL_D];
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            const int k = out.pos(min(i0 + 4 * j, M - 1));
            kk[j] = k;
            r[j] = in.load(k);
            av[j] = ast[k * 16 + s];
            bx[j] = bst[(k + 1) * 16 + nx0];
            by[j] = bst[(k + 1) * 16 + nx1];
        }
#pragma unroll
        for (int j = 0; j < LL_D; ++j) {
            const int i = i0 + 4 * j, k = kk[j];
            if (!__any(i < M)) break;   // the groups run different i: wave-level exit
            double iA, iB;
            in.sums(r[j], iA, iB);
            const float gl = gamma_lane(iA, iB, r[j].v.z, r[j].v.w, s & 7);
            float app[4];
#pragma unroll
            for (int inp = 0; inp < 4; ++inp) {
                const float gv = __shfl(gl, L.base + L.gi[inp]);
                const float t = (av[j] + (L.gn[inp] ? -gv : gv)) + ((inp == 0 || inp == 3) ? bx[j] : by[j]);
                app[inp] = fmaxf(NEG, t);
            }
            row_max16x4(app);
            const float pA0 = app[0] > app[1] ? app[0] : app[1], pA1 = app[2] > app[3] ? app[2] : app[3];
            const float pB0 = app[0] > app[2] ? app[0] : app[2], pB1 = app[1] > app[3] ? app[1] : app[3];
            double x = ((double)(pA0 - pA1) - iA) * sf, y = ((double)(pB0 - pB1) - iB) * sf;
            x = x > 300.0 ? 300.0 : x;
            x = x < -300.0 ? -300.0 : x;
            y = y > 300.0 ? 300.0 : y;
            y = y < -300.0 ? -300.0 : y;
            if (i < M) out.store(k, x, y, r[j].v.x, r[j].v.y);
        }
    }
    ll_sync();
}

// DVBRCS2_Turbo.decode (:464-537), one codeword per wave (block).
__global__ __launch_bounds__(WAVE) void k_turbo_decode_lowlat(LLArgs p, const int *__restrict__ perm,
                                                              const int *__restrict__ inv) {
    extern __shared__ int ll_lds[];   // [3][N]: perm, inv_perm, the used-position list
    const int lane = threadIdx.x, grp = lane >> 4;
    const long cw = blockIdx.x;
    if (cw >= p.B) return;
    const SplLane L = spl_lane(lane);
    const int N = p.N;
    const long tile = cw / WAVE;
    const int cwl = (int)(cw % WAVE);
    const float *base = p.planes + tile * tile_floats(N);
    const float4 *X = reinterpret_cast<const float4 *>(base);
    const float2 *Z = reinterpret_cast<const float2 *>(base + (long)N * WAVE * 4);
    double2 *P1 = p.ws + cw * ll_ws_elems(N), *Le2 = P1 + N, *Le1 = Le2 + N;
    float *ast = p.st + cw * ll_st_elems(N), *bst = ast + (N + 1) * 16;
    lds_int *sperm = (lds_int *)ll_lds, *sinv = sperm + N, *sused = sinv + N;
    for (int k = lane; k < N; k += WAVE) {
        sperm[k] = perm[k];
        sinv[k] = inv[k];
        if (k < p.n_used) sused[k] = p.ulist[k];
        Le2[k] = make_double2(0.0, 0.0);   // the first iteration's a-priori (:490-491)
    }
    ll_sync();
    for (int it = 0; it < p.iters; ++it) {
        const double sf = it < p.iters - 1 ? 0.7 : 1.0;   // :496
        const bool last = it == p.iters - 1;
        ll_siso(LLIn1{X, Le2, sinv, cwl}, LLOut1{P1, last ? Le1 : nullptr, sused, p.n_used}, N, ast, bst, L, grp,
                sf);
        ll_siso(LLIn2{Z, P1, sperm, cwl}, LLOut2{Le2}, N, ast, bst, L, grp, sf);
    }
    // hard decision (:526-537): L = (Lc + La) + Le1, La = Le2[inv_perm]; lane l takes k = l, l + 64, ...
    for (int k = lane; k < N; k += WAVE) {
        const float4 x = X[(long)k * WAVE + cwl];
        const double2 la = Le2[sinv[k]], le = Le1[k];
        const double fa = ((double)x.x + la.x) + le.x;
        const double fb = ((double)x.y + la.y) + le.y;
        *reinterpret_cast<int2 *>(p.bits + cw * 2 * N + 2 * k) = make_int2(fa < 0.0 ? 1 : 0, fb < 0.0 ? 1 : 0);
        if (p.lfinal) *reinterpret_cast<double2 *>(p.lfinal + cw * 2 * N + 2 * k) = make_double2(fa, fb);
    }
}

}  // namespace tdec
