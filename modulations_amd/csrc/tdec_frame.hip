// tdec_frame.hip -- the FRAME decoder (max-log): ONE CODEWORD PER WORKGROUP.
//
// The per-call paths of the reference -- DVBRCS2_Turbo.decode() once per frame
// (test.py:81) and bcjr_max_log_map() once per call (dvb_rcs2_turbo.py:116-281)
// -- are latency problems: one codeword, 16 (or 1) SISOs, each a chain of
// ~2N dependent trellis steps.  Here a 512-thread workgroup owns the codeword
// and everything lives in LDS (alpha / beta stores, the pair-maxima table, the
// extrinsic planes, the interleaver tables).  One SISO is three phases,
// separated by workgroup barriers:
//
//  P  branch metrics, position-parallel (every thread one position): the
//     reference's f64 gamma (:127-160), rounded to f32, reduced to the 8 pair
//     maxima a recursion step reads, into an LDS table.
//  R  the recursions: wave 0 runs alpha, wave 1 beta (:162-230), each on 4
//     16-lane groups, one trellis state per lane.
//       * No cross-lane permute on the chain.  State ns has predecessors
//         rotr(ns) and rotr(ns)^8 (4-bit rotations: ns = ((s<<1)&14)|dk), so
//         with a TIME-VARYING labelling -- lane l holds state rotl^t(l) at step
//         t (beta: rotr^t(rev(l))) -- one predecessor is the lane itself and
//         the other is lane l ^ (8 >> (t % 4)): a DPP move (row_ror:8, two
//         bank-masked row shifts, quad_perm).  The state-0 normalisation reads
//         lane 0 of the row (row_newbcast:0; state 0 is always lane 0).  A step
//         is DPP, two adds, max3, DPP, subtract: no LDS round trip.
//       * Segments, exact.  The 4 groups of a wave take 4 segments of the
//         block.  Segment 0 starts from the reference's zero vector; the others
//         start from zero as a guess, then re-run from their predecessor's true
//         end vector until their vector EQUALS the stored one (IEEE ==): from
//         there the stored trajectory is the same deterministic f32 map of the
//         same vector, so it is the reference's (the merge argument of
//         DESIGN §3 item 2).  A segment that reaches its end without merging
//         hands its new end vector to the next one (rounds until none changes:
//         at most 4).  The reference's second pass (from alpha1[N] / beta1[0])
//         is the same machinery started at segment 0.  Every stored vector is
//         therefore the reference's alpha2 / beta2, bit for bit.
//  E  the extrinsic (:232-281), position-parallel, from the stored alpha2[k],
//     beta2[k+1] and the recomputed branch metrics (extrinsic<0>, the per-lane
//     decoder's code).
// Same f32 / f64 operations as the reference everywhere; maxima are order-free
// (fmaxf drops a NaN as the strict `>` does; only the sign of an exact zero can
// differ, compared with IEEE ==).  tests/test_gpu_frame.py.
#include <type_traits>

namespace tdec {

constexpr int FR_WAVES = 8;
constexpr int FR_BLOCK = FR_WAVES * WAVE;
// Waves per direction in the recursions: 1 or 2 (WPD, chosen per block length by
// tdec_api.hip fr_wpd; see fr_recursion_x).  Two measured faster than one at N = 752
// (profiles/r04e/ab_frame_*, decode of N = 752 r = 1/2: 0.30 vs 0.34 ms at B = 1,
// 0.36 vs 0.38 ms at B = 64, 1.40 vs 1.50 ms at B = 1 024).  Four waves per direction
// (16 segments) halve phase A but need 5.1 rounds per SISO instead of 2.8 and lose:
// 0.36 vs 0.29 ms at B = 1, 1.80 vs 1.39 ms at B = 1 024 (profiles/r04m/).
constexpr int FR_WPD_MAX = 2;
constexpr int FR_NSEG_MAX = 8;   // segments per direction at most (4 per wave)
// Segments per direction = N / FR_LMIN (at least 1, at most the
// P the waves provide), the steps split evenly over them in whole 4-step blocks.
// A segment shorter than the recursions' typical merge depth (~40 steps) rarely
// merges in its first re-run, so the rounds hand end vectors down a chain of
// segments: at N = 48 the even split (8-step segments) made every SISO ~17 us of
// rounds and barriers where one 48-step segment is two serial passes (round 5's
// first rule, a floor of 48 steps, profiles/r05c/: decode() per frame N = 48 0.291 ->
// 0.148 ms).  The floor left N = 64 as 48 + 16 steps; splitting evenly with at
// least 32 steps per segment gives 32 + 32 (one wave per direction,
// profiles/r05/lmin_wpd1/: N = 64 0.150 -> 0.123 ms) and the same segments at
// every other block size.
constexpr int FR_LMIN = 32;
__host__ __device__ constexpr int fr_seg_len(int N, int P) {
    int n = N / FR_LMIN;
    n = n < 1 ? 1 : (n > P ? P : n);
    return (N + 4 * n - 1) / (4 * n) * 4;
}
typedef __attribute__((address_space(3))) char lds_b;   // byte-addressed LDS

__device__ __forceinline__ float lds_ld(const lds_b *p) { return *(const lds_f1 *)p; }
__device__ __forceinline__ void lds_st(lds_b *p, float v) { *(lds_f1 *)p = v; }

// ---- LDS layout (bytes) ------------------------------------------------------------
// ev [2][8][16] f32 segment end vectors (+ 64 B of round control), sink [2][512 B] (stores of idle groups),
// st_a [N+1][16] f32 (alpha[k] at row k), st_b [N+1][16] (beta[k] at row k), pmt
// [N][8] f32 pair maxima; the decoder adds p1, le2 [N] double2 and perm, inv
// [N] int.  The recursions read up to 16 rows past pmt / st in either
// direction (prefetch; values unused): the arrays before st_a and the tail pad
// keep those reads inside the allocation.
struct FrLds {
    int st_a, st_b, pmt, ev, sink, p1, le2, perm, inv, total;
};
// le2_global (the decoder at N > 805, where the LDS plan is 8.5 KB over at N = 848):
// decoder 2's extrinsic plane Le2 lives in the workgroup's own [N] double2 row of
// global scratch (L2-resident) instead of LDS.
__host__ __device__ constexpr FrLds fr_lds(int N, bool dec, bool le2_global = false) {
    FrLds L{};
    int o = 0;
    L.ev = o;   o += 2 * FR_NSEG_MAX * 64 + 64;   // 2 directions x 8 (16) segments; + the cross-wave rounds' control words
    L.sink = o; o += 2 * 512;
    L.st_a = o; o += (N + 1) * 64;
    L.st_b = o; o += (N + 1) * 64;
    L.pmt = o;  o += N * 32;
    L.p1 = L.le2 = L.perm = L.inv = o;
    if (dec) {
        L.p1 = o;    o += N * 16;
        L.le2 = o;   o += le2_global ? 0 : N * 16;
        L.perm = o;  o += N * 4;
        L.inv = o;   o += N * 4;
    }
    L.total = o + 512;   // tail: the alpha wave's reads past pmt
    return L;
}
constexpr int FR_LDS_MAX = 160 * 1024;

// ---- lane labelling ------------------------------------------------------------------
__host__ __device__ constexpr int rotl4(int x, int r) {
    r &= 3;
    return ((x << r) | (x >> (4 - r))) & 15;
}
__host__ __device__ constexpr int rotr4(int x, int r) { return rotl4(x, 4 - (r & 3)); }
__host__ __device__ constexpr int rev4(int x) { return ((x & 1) << 3) | ((x & 2) << 1) | ((x & 4) >> 1) | ((x & 8) >> 3); }
// pair-maxima index (pair_max: class A^B * 4 + 2W + Y) of the branch pair p -> ns
__host__ __device__ constexpr int pair_ix(int p, int ns) {
    for (int inp = 0; inp < 4; ++inp)
        if (t_next(p, inp) == ns) return ((((inp >> 1) ^ inp) & 1) << 2) | (t_ow(p, inp) << 1) | t_oy(p, inp);
    return 0;
}

// Per-lane constants of a recursion lane, for the 4 phases ph = t % 4 of a step.
// lbl[ph]: state of the lane's element of the vector entering a phase-ph step
// (alpha: rotl^ph(l); beta: rotr^ph(rev(l))); soff: its byte offset in a store row
// plus the row step from the block's first row; poff: the pm-table offsets of
// the lane's own pair and its partner's (lane l ^ (8 >> ph)) pair, likewise.
template <int DIR> struct FrLane {
    int lbl[4];
    int soff[4];
    int poff[4][2];
};
template <int DIR> __device__ __forceinline__ FrLane<DIR> fr_lane(int l) {
    FrLane<DIR> L;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
        int in, a, b;
        if (DIR == 0) {   // alpha: produces ns = rotl^(ph+1)(l) from in = rotr(ns) (self) and in ^ 8 (partner)
            in = rotl4(l, ph);
            const int ns = rotl4(l, ph + 1);
            a = pair_ix(in, ns);
            b = pair_ix(in ^ 8, ns);
        } else {          // beta: produces s = rotr^(ph+1)(rev l) from its successors in = rotl(s) and in ^ 1
            in = rotr4(rev4(l), ph);
            const int s = rotr4(rev4(l), ph + 1);
            a = pair_ix(s, in);
            b = pair_ix(s, in ^ 1);
        }
        const int dir = DIR ? -1 : 1;
        L.lbl[ph] = in;
        L.soff[ph] = dir * 64 * ph + 4 * in;
        L.poff[ph][0] = dir * 32 * ph + 4 * a;
        L.poff[ph][1] = dir * 32 * ph + 4 * b;
    }
    return L;
}

// one trellis step (:165-179 / :203-213 with pair maxima): max over the two branch
// pairs into the lane's new state, from -1e9, minus state 0 (lane 0 of the row).
// The partner's add and the normalisation are DPP forms of the VALU ops themselves
// (v_add_f32_dpp: partner + po; v_subrev_f32_dpp: n - n[lane 0]), not a DPP move
// feeding them -- 2 fewer instructions on the serial chain (3 in the xor-4 phase).
// Same IEEE operations, so the same bits.  The s_nop 1 covers the VALU-write ->
// DPP-read hazard (2 wait states), which the compiler does not track through
// inline asm.  Measured 0.34 vs 0.35 ms per decode at B = 1, 1.50 vs 1.52 ms at B =
// 1 024 (profiles/r04e/ab_frame_*).  (Every lane forming state 0's new value itself
// instead of waiting for lane 0's through a second DPP move measured slower: 0.39
// vs 0.34 ms.)
template <int PH> __device__ __forceinline__ float fr_partner_add(float v, float po) {
    float y;
    if constexpr (PH == 0)
        asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 row_ror:8 row_mask:0xf bank_mask:0xf" : "=v"(y) : "v"(v), "v"(po));
    else if constexpr (PH == 1)
        asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
            "v_add_f32_dpp %0, %1, %2 row_shr:4 row_mask:0xf bank_mask:0xa"
            : "=&v"(y) : "v"(v), "v"(po));
    else if constexpr (PH == 2)
        asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "=v"(y) : "v"(v), "v"(po));
    else
        asm("s_nop 1\n\tv_add_f32_dpp %0, %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(y) : "v"(v), "v"(po));
    return y;
}
template <int PH> __device__ __forceinline__ float fr_step(float v, float ps, float po) {
    const float y = fr_partner_add<PH>(v, po);
    const float n = fmaxf(fmaxf(NEG, v + ps), y);
    float r;
    asm("s_nop 1\n\tv_subrev_f32_dpp %0, %1, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(n));
    return r;
}

// log-MAP (ALGO 1): the same step with max* (jac, tdec_kernels.hip) over the lane's
// own pair value and its partner's in place of max3 with -1e9 (alpha_step /
// beta_step's jac(x0, y0) over a state's two predecessor / successor classes: jac
// is symmetric, so which of the two the lane holds does not matter), then the
// same state-0 normalisation.
template <int PH> __device__ __forceinline__ float fr_step_lm(float v, float ps, float po) {
    const float y = fr_partner_add<PH>(v, po);
    const float n = jac(v + ps, y);
    float r;
    asm("s_nop 1\n\tv_subrev_f32_dpp %0, %1, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(n));
    return r;
}
template <int ALGO, int PH> __device__ __forceinline__ float fr_step_a(float v, const float (&c)[2]) {
    if constexpr (ALGO == 1) return fr_step_lm<PH>(v, c[0], c[1]);
    else return fr_step<PH>(v, c[0], c[1]);
}

// Fast blocks of 8 steps (two labelling periods), max-log as one asm sequence: the
// same instructions as fr_step / lds_st (own add, DPP partner add, v_max3 with -1e9,
// DPP normalisation by lane 0), so the same bits, with each store and the next
// step's own add placed in the DPP read-after-write hazard slots instead of s_nop,
// no per-step s_waitcnt (the stores are not waited on here; the compiler's later
// waits count only its own LDS operations, which retire in order before these, so
// they stay conservative), and the block's control (run-mask and end tests, the
// merge compare, address updates, the next block's pair-maxima loads) paid once per
// 8 steps.  a[ph]: LDS byte address of the vector entering step ph of the block's
// LOWER-addressed half (alpha: steps 0-3 at +0, 4-7 at +256; beta, whose rows
// descend: steps 0-3 at +256, 4-7 at +0), c[j]: step j's own / partner pair maxima.
// (4-step asm blocks: 0.28 vs 0.29 ms per decode at B = 1 against C++ steps,
// profiles/r04s/; 8-step blocks faster again, round 5.)  log-MAP runs the same
// 8-step blocks as C++ steps (profiles/r05/frame_lm8/: log-MAP decode() per frame
// N = 752 r = 1/2 1.085 -> 0.916 ms, N = 48 0.200 -> 0.178 ms; same bits).
#define FR8_STEP0(A, OFF, CO, CP, NOP)                                                          \
    "ds_write_b32 %[" A "], %[v] offset:" OFF "\n\t"                                          \
    "v_add_f32 %[u], %[v], %[" CO "]\n\t" NOP                                                 \
    "v_add_f32_dpp %[t], %[v], %[" CP "] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"            \
    "v_max3_f32 %[n], %[u], %[neg], %[t]\n\t"                                                 \
    "s_nop 1\n\t"                                                                             \
    "v_subrev_f32_dpp %[v], %[n], %[n] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
#define FR8_STEP1(A, OFF, CO, CP)                                                               \
    "ds_write_b32 %[" A "], %[v] offset:" OFF "\n\t"                                          \
    "v_add_f32 %[u], %[v], %[" CO "]\n\t"                                                     \
    "v_add_f32_dpp %[t], %[v], %[" CP "] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"            \
    "v_add_f32_dpp %[t], %[v], %[" CP "] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"            \
    "v_max3_f32 %[n], %[u], %[neg], %[t]\n\t"                                                 \
    "s_nop 1\n\t"                                                                             \
    "v_subrev_f32_dpp %[v], %[n], %[n] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
#define FR8_STEPQ(A, OFF, CO, CP, QP)                                                           \
    "ds_write_b32 %[" A "], %[v] offset:" OFF "\n\t"                                          \
    "v_add_f32 %[u], %[v], %[" CO "]\n\t"                                                     \
    "v_add_f32_dpp %[t], %[v], %[" CP "] quad_perm:" QP " row_mask:0xf bank_mask:0xf\n\t"     \
    "v_max3_f32 %[n], %[u], %[neg], %[t]\n\t"                                                 \
    "s_nop 1\n\t"                                                                             \
    "v_subrev_f32_dpp %[v], %[n], %[n] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
#define FR8_BODY(O0, O1)                                                                        \
    FR8_STEP0("a0", O0, "c00", "c01", "s_nop 1\n\t")                                          \
    FR8_STEP1("a1", O0, "c10", "c11")                                                         \
    FR8_STEPQ("a2", O0, "c20", "c21", "[2,3,0,1]")                                            \
    FR8_STEPQ("a3", O0, "c30", "c31", "[1,0,3,2]")                                            \
    FR8_STEP0("a0", O1, "c40", "c41", "")                                                     \
    FR8_STEP1("a1", O1, "c50", "c51")                                                         \
    FR8_STEPQ("a2", O1, "c60", "c61", "[2,3,0,1]")                                            \
    FR8_STEPQ("a3", O1, "c70", "c71", "[1,0,3,2]")                                            \
    "s_nop 1"
template <int DIR>
__device__ __forceinline__ void fr_block8_asm(float &v, const float (&c)[8][2], unsigned a0, unsigned a1, unsigned a2,
                                              unsigned a3) {
    float t, u, n;
#define FR8_OPERANDS                                                                                                  \
    : [v] "+v"(v), [t] "=&v"(t), [u] "=&v"(u), [n] "=&v"(n)                                                          \
    : [a0] "v"(a0), [a1] "v"(a1), [a2] "v"(a2), [a3] "v"(a3), [c00] "v"(c[0][0]), [c01] "v"(c[0][1]),                \
      [c10] "v"(c[1][0]), [c11] "v"(c[1][1]), [c20] "v"(c[2][0]), [c21] "v"(c[2][1]), [c30] "v"(c[3][0]),            \
      [c31] "v"(c[3][1]), [c40] "v"(c[4][0]), [c41] "v"(c[4][1]), [c50] "v"(c[5][0]), [c51] "v"(c[5][1]),            \
      [c60] "v"(c[6][0]), [c61] "v"(c[6][1]), [c70] "v"(c[7][0]), [c71] "v"(c[7][1]), [neg] "s"(NEG)                 \
    : "memory"
    if constexpr (DIR == 0) asm volatile(FR8_BODY("0", "256") FR8_OPERANDS);
    else asm volatile(FR8_BODY("256", "0") FR8_OPERANDS);
#undef FR8_OPERANDS
}
#undef FR8_BODY
#undef FR8_STEPQ
#undef FR8_STEP1
#undef FR8_STEP0

// lanes of the 16-lane groups whose 16 bits of m are all set
// A wave-uniform 64-bit value the compiler cannot prove uniform (it came from LDS or
// a lane-dependent expression), moved to SGPRs: the round loop's control flow
// then stays scalar (branches on SCC) instead of divergent exec-mask loops with
// the masks held in VGPRs.
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x), hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned long long grp_all16(unsigned long long m) {
    unsigned long long r = 0;
#pragma unroll
    for (int g = 0; g < 4; ++g)
        if (((m >> (16 * g)) & 0xFFFFull) == 0xFFFFull) r |= 0xFFFFull << (16 * g);
    return r;
}

struct FrRec {
    lds_b *st;     // this direction's store
    lds_b *pmt;    // pair maxima [N][8]
    lds_b *ev;     // [4][16] end vectors of this direction
    lds_b *sink;   // 512 B
    int N;
};

// TDEC_FR_STATS (measurement builds): 1 = block / round counters and phase timers,
// 2 = the phase timers alone (no atomics inside the recursion loops)
#ifndef TDEC_FR_STATS
#define TDEC_FR_STATS 0
#endif
#if TDEC_FR_STATS
__device__ unsigned long long g_fr_stats[8];   // blocks run: phase A, fix-up, pass 2; rounds: fix-up, pass 2;
                                               // s_memrealtime ticks (100 MHz) of phases P, R, E (thread 0)
#endif

// One round of the groups in `run` (wave-uniform lane mask), each from its start
// vector v over its segment [u0, u0 + len) of the direction's step order:
// stores every vector entering a step; with CMP, stops a group at the first
// block start where its vector equals the stored one (merged).  Returns the
// lanes of the groups that reached their segment's end (their end vector, the
// one entering step u0 + len, is in ev[g]).
template <int DIR, bool CMP, int ALGO = 0>
__device__ __forceinline__ unsigned long long fr_round(const FrRec &R, const FrLane<DIR> &L, int g, int lane, int u0,
                                                       int len, unsigned long long run, float v, int stat) {
    const int N = R.N;
    run = uni64(run);
    // byte offsets of the rows of step U: store row (alpha[U] / beta[N - U]) and pm row (position)
    auto srow = [&](int U) { return (DIR ? N - U : U) * 64; };
    auto prow = [&](int U) { return (DIR ? N - 1 - U : U) * 32; };
    unsigned long long reached = 0;
    float cmpv = 0.0f, cmpn = 0.0f;
    if constexpr (CMP) cmpv = lds_ld(R.st + srow(u0) + L.soff[0]);
    {
        // 8-step blocks: the pair maxima of 8 steps from the block's two row halves
        // (alpha: rows U, U + 4 ascending; beta: its rows descend, so the lower half
        // U + 4 is the base and U sits 4 rows above it)
        auto load8 = [&](int U, float (&c)[8][2]) {
            const lds_b *pb = R.pmt + prow(DIR ? U + 4 : U);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int ph = j & 3, h = j >> 2, hoff = DIR ? (h ? 0 : 128) : (h ? 128 : 0);
                c[j][0] = lds_ld(pb + hoff + L.poff[ph][0]);
                c[j][1] = lds_ld(pb + hoff + L.poff[ph][1]);
            }
        };
        auto block8 = [&](int u, float (&c)[8][2], float (&n)[8][2], float &cv, float &cn) -> bool {
            if constexpr (CMP) run &= ~grp_all16(__ballot(v == cv));   // merged: the rest is stored already
            if (!run) return false;
            const int U = u0 + u;
            load8(U + 8, n);   // the next block's (rows past the end are read, unused)
            if constexpr (CMP) cn = lds_ld(R.st + srow(U + 8) + L.soff[0]);
            const bool rl = (run >> lane) & 1;
            if (!(__ballot(u + 8 >= len) & run)) {   // every running group has steps after this block
                // idle groups store into their sink row: alpha and beta both at [0, 508)
                lds_b *const sr = rl ? R.st + srow(DIR ? U + 4 : U) : R.sink + (DIR ? 192 : 0);
                if constexpr (ALGO == 0) {
                    fr_block8_asm<DIR>(v, c, (unsigned)(uintptr_t)(sr + L.soff[0]),
                                       (unsigned)(uintptr_t)(sr + L.soff[1]), (unsigned)(uintptr_t)(sr + L.soff[2]),
                                       (unsigned)(uintptr_t)(sr + L.soff[3]));
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int h = j >> 2, hoff = DIR ? (h ? 0 : 256) : (h ? 256 : 0);
                        lds_st(sr + hoff + L.soff[j & 3], v);
                        const float c4[2] = {c[j][0], c[j][1]};
                        switch (j & 3) {
                        case 0: v = fr_step_a<ALGO, 0>(v, c4); break;
                        case 1: v = fr_step_a<ALGO, 1>(v, c4); break;
                        case 2: v = fr_step_a<ALGO, 2>(v, c4); break;
                        default: v = fr_step_a<ALGO, 3>(v, c4); break;
                        }
                    }
                }
            } else {   // some group ends in this block: per-step bounds, end vector captured
                lds_b *const evg = R.ev + g * 64;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int uu = u + j;
                    lds_b *const rw = R.st + srow(U + (j & 4));
                    const float c4[2] = {c[j][0], c[j][1]};
                    if (rl && uu < len) lds_st(rw + L.soff[j & 3], v);
                    float vn;
                    switch (j & 3) {
                    case 0: vn = fr_step_a<ALGO, 0>(v, c4); break;
                    case 1: vn = fr_step_a<ALGO, 1>(v, c4); break;
                    case 2: vn = fr_step_a<ALGO, 2>(v, c4); break;
                    default: vn = fr_step_a<ALGO, 3>(v, c4); break;
                    }
                    if (rl && uu == len - 1) lds_st(evg + 4 * L.lbl[(j + 1) & 3], vn);
                    v = vn;
                }
                const unsigned long long ended = __ballot(u + 8 >= len) & run;
                reached |= ended;
                run &= ~ended;
            }
            return true;
        };
        float qc[8][2], qn[8][2];
        load8(u0, qc);
        for (int u = 0;; u += 16) {
            if (!block8(u, qc, qn, cmpv, cmpn)) break;
            if (!block8(u + 8, qn, qc, cmpn, cmpv)) break;
        }
    }
    (void)stat;
    return reached;
}

// Both passes of one direction (alpha: :162-197, beta: :199-230) by one wave.
// On exit row k of R.st holds alpha2[k] (k < N) / beta2[k] (k >= 1).
template <int DIR, int ALGO = 0> __device__ void fr_recursion(const FrRec &R, int lane) {
    const int l = lane & 15, g = lane >> 4;
    const FrLane<DIR> L = fr_lane<DIR>(l);
    const int N = R.N;
    const int Ls = fr_seg_len(N, 4);        // segment length (a multiple of 4)
    const int nseg = (N + Ls - 1) / Ls;     // 1..4
    const int len = max(0, min(Ls, N - g * Ls)), u0 = len ? g * Ls : 0;   // empty segments never run
    const unsigned long long all = nseg == 4 ? ~0ull : (1ull << (16 * nseg)) - 1;
    const lds_b *src = R.ev + (g == 0 ? nseg - 1 : g - 1) * 64 + 4 * L.lbl[0];   // the start of a re-run
    // pass 1, phase A: every segment from zero (segment 0: the reference's start)
    unsigned long long reached = fr_round<DIR, false, ALGO>(R, L, g, lane, u0, len, all, 0.0f, 0);
    unsigned long long dirty = (reached << 16) & all;
    // The first re-run round also starts the reference's second pass SPECULATIVELY:
    // group 0 (idle in the re-runs) runs from the last segment's phase-A end
    // vector.  If that round leaves pass 1 complete and the last segment's end
    // unchanged, that start was alpha1[N] / beta1[0] and the second pass goes on
    // from this round's state; otherwise the second pass restarts below from the
    // verified end vector.  (Merging against whatever segment 0 holds is exact
    // either way: a stored segment is always one consistent trajectory.)
    const unsigned long long G0 = 0xFFFFull, GL = 0xFFFFull << (16 * (nseg - 1));
    bool spec = false, broken = false;
    if (dirty) {
#if TDEC_FR_STATS == 1
        if (lane == 0) atomicAdd(&g_fr_stats[3], 1ull);
#endif
        reached = fr_round<DIR, true, ALGO>(R, L, g, lane, u0, len, dirty | G0, lds_ld(src), 1);
        const unsigned long long r1 = reached & ~G0;
        spec = !(r1 & GL);              // the last segment's end vector did not change
        dirty = (r1 << 16) & all;
        if (!dirty && spec) {
            dirty = (reached & G0) << 16 & all;   // pass 1 done: the second pass continues
        } else {
            spec = false;
            // if group 0 ran to its end, ev[0] and segment 0 hold the speculative
            // trajectory while segment 1 still holds the pass-1 one: the chain of
            // end vectors is broken at segment 0 until segment 1 re-runs
            broken = (reached & G0) != 0;
        }
        // the remaining pass-1 rounds
        while (!spec && dirty) {
#if TDEC_FR_STATS == 1
            if (lane == 0) atomicAdd(&g_fr_stats[3], 1ull);
#endif
            reached = fr_round<DIR, true, ALGO>(R, L, g, lane, u0, len, dirty, lds_ld(src), 1);
            dirty = (reached << 16) & all;
        }
    }
    // the second pass (from alpha1[N] / beta1[0] at segment 0) unless the
    // speculative start was right, then its remaining rounds
    if (!spec) {
#if TDEC_FR_STATS == 1
        if (lane == 0) atomicAdd(&g_fr_stats[4], 1ull);
#endif
        reached = fr_round<DIR, true, ALGO>(R, L, g, lane, u0, len, G0, lds_ld(src), 2);
        dirty = ((reached & G0) || broken) ? (G0 << 16) & all : 0ull;
    }
    while (dirty) {
#if TDEC_FR_STATS == 1
        if (lane == 0) atomicAdd(&g_fr_stats[4], 1ull);
#endif
        reached = fr_round<DIR, true, ALGO>(R, L, g, lane, u0, len, dirty, lds_ld(src), 2);
        dirty = (reached << 16) & all;
    }
}

// ---- WPD 2: 8 segments per direction on two waves each -------------------------------------
// The same rounds as fr_recursion, with the segments of one direction spread over
// two waves (alpha: waves 0-1, beta: waves 2-3), so each round is a workgroup step:
// every wave (the idle ones too) passes three barriers per round -- starts read
// before any end vector is written, rounds run, thread 0 advances both
// directions' round state from the segments that reached their end.
struct FrCtl {
    unsigned dirty[2], reached[2], state[2], broken[2], cmp[2];
};
enum { FR_A = 0, FR_FIX1 = 1, FR_FIXN = 2, FR_P2S = 3, FR_P2 = 4 };
template <int ALGO = 0> __device__ void fr_recursion_x(lds_b *sm, const FrLds &Lo, int N, int wave, int lane) {
    volatile __attribute__((address_space(3))) FrCtl *ctl =
        (volatile __attribute__((address_space(3))) FrCtl *)(sm + Lo.ev + 2 * FR_NSEG_MAX * 64);
    constexpr int WPDX = 2;   // waves per direction
    const int Ls = fr_seg_len(N, 4 * WPDX);   // segment length (a multiple of 4)
    const int nseg = (N + Ls - 1) / Ls;     // 1..4 * WPDX
    const unsigned all = (1u << nseg) - 1;
    const bool rw = wave < 2 * WPDX;
    const int dir = wave / WPDX, wl = wave % WPDX, l = lane & 15, g = lane >> 4, G = 4 * wl + g;
    const int len = max(0, min(Ls, N - G * Ls)), u0 = len ? G * Ls : 0;
    if (threadIdx.x == 0)
        for (int d = 0; d < 2; ++d) {
            ctl->dirty[d] = all;
            ctl->reached[d] = 0u;
            ctl->state[d] = FR_A;
            ctl->broken[d] = 0u;
            ctl->cmp[d] = 0u;
        }
    FrLane<0> La = fr_lane<0>(l);
    FrLane<1> Lb = fr_lane<1>(l);
    const FrRec Ra{sm + Lo.st_a, sm + Lo.pmt, sm + Lo.ev, sm + Lo.sink, N};
    const FrRec Rb{sm + Lo.st_b, sm + Lo.pmt, sm + Lo.ev + FR_NSEG_MAX * 64, sm + Lo.sink + 512, N};
    __syncthreads();
#if TDEC_FR_STATS == 2
    // timers-only build: [0] ticks of round 0 (phase A), [1] of the later rounds,
    // [2] rounds, [3] ticks wave 0 spends inside fr_round, [4] ticks of wave 0's phase A
    unsigned long long t_round = __builtin_amdgcn_s_memrealtime();
    int n_round = 0;
#endif
    for (;;) {
        const unsigned dm = rw ? ctl->dirty[dir] : 0u, cmp = rw ? ctl->cmp[dir] : 0u;
        const bool any = (ctl->dirty[0] | ctl->dirty[1]) != 0u;
        unsigned long long run = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if ((dm >> (4 * wl + q)) & 1u) run |= 0xFFFFull << (16 * q);
        float v = 0.0f;
        if (rw && cmp) {
            const int src = G == 0 ? nseg - 1 : G - 1;
            v = lds_ld((dir ? Rb.ev : Ra.ev) + src * 64 + 4 * (dir ? Lb.lbl[0] : La.lbl[0]));
        }
        __syncthreads();   // every start is read before any end vector of this round is written
        if (!any) break;
        if (rw && run) {
#if TDEC_FR_STATS == 2
            const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
#endif
            unsigned long long r;
            const int stat = cmp ? (ctl->state[dir] == FR_P2 || ctl->state[dir] == FR_P2S ? 2 : 1) : 0;
            if (dir == 0) r = cmp ? fr_round<0, true, ALGO>(Ra, La, G, lane, u0, len, run, v, stat)
                                  : fr_round<0, false, ALGO>(Ra, La, G, lane, u0, len, run, v, stat);
            else r = cmp ? fr_round<1, true, ALGO>(Rb, Lb, G, lane, u0, len, run, v, stat)
                         : fr_round<1, false, ALGO>(Rb, Lb, G, lane, u0, len, run, v, stat);
            unsigned bits = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((r >> (16 * q)) & 1ull) bits |= 1u << (4 * wl + q);
            if (lane == 0 && bits) atomicOr((unsigned *)&ctl->reached[dir], bits);
#if TDEC_FR_STATS == 2
            if (threadIdx.x == 0) {
                const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - tw;
                atomicAdd(&g_fr_stats[3], dt);
                if (n_round == 0) atomicAdd(&g_fr_stats[4], dt);
            }
#endif
        }
        __syncthreads();
        if (threadIdx.x == 0)
            for (int d = 0; d < 2; ++d) {
                const unsigned r = ctl->reached[d];
                unsigned dirty = 0;
                switch (ctl->state[d]) {
                case FR_A: {   // phase A done: re-runs + the speculative second pass on segment 0
                    const unsigned d1 = (r << 1) & all;
                    if (d1) {
                        dirty = d1 | 1u;
                        ctl->state[d] = FR_FIX1;
                    } else {
                        dirty = 1u;
                        ctl->state[d] = FR_P2S;
                    }
                    ctl->cmp[d] = 1u;
                    break;
                }
                case FR_FIX1: {
                    const unsigned r1 = r & ~1u, dd = (r1 << 1) & all;
                    const bool spec = !(r1 & (1u << (nseg - 1)));
                    if (!dd && spec) {
                        dirty = ((r & 1u) << 1) & all;
                        ctl->state[d] = FR_P2;
                    } else {
                        ctl->broken[d] = r & 1u;
                        if (dd) {
                            dirty = dd;
                            ctl->state[d] = FR_FIXN;
                        } else {
                            dirty = 1u;
                            ctl->state[d] = FR_P2S;
                        }
                    }
                    break;
                }
                case FR_FIXN: {
                    const unsigned dd = (r << 1) & all;
                    if (dd) {
                        dirty = dd;
                    } else {
                        dirty = 1u;
                        ctl->state[d] = FR_P2S;
                    }
                    break;
                }
                case FR_P2S:
                    dirty = ((r & 1u) || ctl->broken[d]) ? 2u & all : 0u;
                    ctl->state[d] = FR_P2;
                    break;
                default:
                    dirty = (r << 1) & all;
                    break;
                }
                if (ctl->dirty[d] == 0u) dirty = 0u;   // a finished direction stays finished
                ctl->dirty[d] = dirty;
                ctl->reached[d] = 0u;
            }
        __syncthreads();
#if TDEC_FR_STATS == 2
        if (threadIdx.x == 0) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            atomicAdd(&g_fr_stats[n_round == 0 ? 0 : 1], now - t_round);
            atomicAdd(&g_fr_stats[2], 1ull);
            t_round = now;
        }
        ++n_round;
#endif
    }
}

// ---- inputs / outputs of one SISO -------------------------------------------------------
// Thread t owns the positions ord[t + j * FR_BLOCK] (j < FR_J) in both position-
// parallel phases of every SISO, so their channel values (In::Raw) are fetched from
// HBM once per kernel and stay in registers (16 P and 16 E phases per decode: a
// global-load round trip per phase otherwise).  The decoder's order puts the
// positions in perm's image first (decoder 1's sparse extrinsic phase is then
// ord[0 .. n_used)); the SISO kernel's order is the identity.
constexpr int FR_J = 2;                    // positions per thread: N <= FR_J * FR_BLOCK = 1024
// get(raw, k): the f64 sums inA = f64(Lc_A) + La_A, inB (:135-136), the parities and Lc.
template <class P> struct FrIn1T {   // decoder 1: planes X = {A, B, W1, Y1}, a-priori Le2[inv_perm[k]] (LDS or global)
    typedef float4 Raw;
    P le2;   // lds_d2 * (LDS) or const double2 * (global scratch)
    const lds_int *inv;
    __device__ __forceinline__ void get(const Raw &x, int k, double &iA, double &iB, double &w, double &y, float &la,
                                        float &lb) const {
        const auto p = le2[inv[k]];
        iA = (double)x.x + p.x;
        iB = (double)x.y + p.y;
        w = x.z;
        y = x.w;
        la = x.x;
        lb = x.y;
    }
};
typedef FrIn1T<const lds_d2 *> FrIn1;
struct FrIn2 {   // decoder 2: planes Z = {W2, Y2}, P1[perm[k]] = f64(Lc) + Le1 (LDS; :507-516)
    typedef float2 Raw;
    const lds_b *p1;
    const lds_int *perm;
    __device__ __forceinline__ void get(const Raw &z, int k, double &iA, double &iB, double &w, double &y, float &la,
                                        float &lb) const {
        const d2v p = *(const lds_d2 *)(p1 + 16 * perm[k]);
        iA = p.x;
        iB = p.y;
        w = z.x;
        y = z.y;
        la = lb = 0.0f;
    }
};
// bcjr_max_log_map's arguments (:116), one row; T = the channel LLRs' dtype
// (float32, or float64: numba's f64 specialisation, sums from unrounded values)
template <typename T> struct FrRowRaw {
    T a, b, w, y;
    double la, lb;
};
template <typename T> struct FrInRow {
    typedef FrRowRaw<T> Raw;
    const T *A, *B, *W, *Y;
    const double *LaA, *LaB;
    __device__ __forceinline__ Raw fetch(int k) const { return Raw{A[k], B[k], W[k], Y[k], LaA[k], LaB[k]}; }
    __device__ __forceinline__ void get(const Raw &r, int, double &iA, double &iB, double &w, double &y, float &la,
                                        float &lb) const {
        iA = (double)r.a + r.la;
        iB = (double)r.b + r.lb;
        w = r.w;
        y = r.y;
        la = lb = 0.0f;
    }
};
struct FrOut1 {  // P1 = f64(Lc) + Le1 for decoder 2 (LDS), Le1 itself in the last iteration (global)
    lds_b *p1;
    double2 *le1;
    int n_used;
    __device__ __forceinline__ int count(int N) const { return le1 ? N : n_used; }   // sparse before the last iteration
    __device__ __forceinline__ void store(int k, double a, double b, float la, float lb) const {
        *(lds_d2 *)(p1 + 16 * k) = d2v{(double)la + a, (double)lb + b};
        if (le1) le1[k] = make_double2(a, b);
    }
};
template <class P> struct FrOut2T {
    P le2;   // lds_d2 * or double2 *
    __device__ __forceinline__ int count(int N) const { return N; }
    __device__ __forceinline__ void store(int k, double a, double b, float, float) const {
        if constexpr (std::is_same<P, double2 *>::value) le2[k] = make_double2(a, b);
        else le2[k] = d2v{a, b};
    }
};
struct FrOutRow {
    double *A, *B;
    __device__ __forceinline__ int count(int N) const { return N; }
    __device__ __forceinline__ void store(int k, double a, double b, float, float) const {
        A[k] = a;
        B[k] = b;
    }
};

// One SISO (:116-281) of the workgroup's codeword.  pos[j]: this thread's positions
// (-1: none), raw[j] their channel values.  Ends with a barrier.
template <int ALGO, int WPD, class In, class Out>
__device__ void fr_siso(const In &in, const Out &out, const int (&pos)[FR_J], const typename In::Raw (&raw)[FR_J],
                        lds_b *sm, const FrLds &Lo, int N, double sf) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    lds_b *pmt = sm + Lo.pmt;
#if TDEC_FR_STATS
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
    // P: pair maxima of every position
#pragma unroll
    for (int j = 0; j < FR_J; ++j) {
        const int k = pos[j];
        if (k < 0) continue;
        double iA, iB, w, y;
        float la, lb;
        in.get(raw[j], k, iA, iB, w, y, la, lb);
        float g[8], pm[2][4];
        gamma_from_sums<ALGO>(iA, iB, w, y, g);
        if constexpr (ALGO == 1) pair_jac(g, pm);   // log-MAP pair values v(wy) + max*(U_c, -U_c)
        else pair_max(g, pm);
        lds_f4 *d = (lds_f4 *)(pmt + 32 * k);
        d[0] = f4v{pm[0][0], pm[0][1], pm[0][2], pm[0][3]};
        d[1] = f4v{pm[1][0], pm[1][1], pm[1][2], pm[1][3]};
    }
    __syncthreads();
#if TDEC_FR_STATS
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
#endif
    // R: alpha on wave 0, beta on wave 1 (WPD 2: alpha on waves 0-1, beta on 2-3)
    if constexpr (WPD == 1) {
        if (wave == 0) fr_recursion<0, ALGO>(FrRec{sm + Lo.st_a, pmt, sm + Lo.ev, sm + Lo.sink, N}, lane);
        else if (wave == 1) fr_recursion<1, ALGO>(FrRec{sm + Lo.st_b, pmt, sm + Lo.ev + FR_NSEG_MAX * 64, sm + Lo.sink + 512, N}, lane);
    } else {
        fr_recursion_x<ALGO>(sm, Lo, N, wave, lane);
    }
    __syncthreads();
#if TDEC_FR_STATS
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
#endif
    // E: extrinsic of every position anyone reads (slots i < M of the order)
    const int M = out.count(N);
#pragma unroll
    for (int j = 0; j < FR_J; ++j) {
        const int k = pos[j];
        if (k < 0 || tid + j * FR_BLOCK >= M) continue;
        double iA, iB, w, y;
        float la, lb;
        in.get(raw[j], k, iA, iB, w, y, la, lb);
        float g[8];
        gamma_from_sums<ALGO>(iA, iB, w, y, g);
        float a[NS], b[NS];
        const lds_f4 *ra = (const lds_f4 *)(sm + Lo.st_a + 64 * k), *rb = (const lds_f4 *)(sm + Lo.st_b + 64 * (k + 1));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f4v x = ra[q], z = rb[q];
            a[4 * q] = x.x, a[4 * q + 1] = x.y, a[4 * q + 2] = x.z, a[4 * q + 3] = x.w;
            b[4 * q] = z.x, b[4 * q + 1] = z.y, b[4 * q + 2] = z.z, b[4 * q + 3] = z.w;
        }
        double leA, leB;
        extrinsic<ALGO>(a, g, b, iA, iB, sf, leA, leB);
        out.store(k, leA, leB, la, lb);
    }
    __syncthreads();
#if TDEC_FR_STATS
    if (tid == 0) {
        const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&g_fr_stats[5], t1 - t0);
        atomicAdd(&g_fr_stats[6], t2 - t1);
        atomicAdd(&g_fr_stats[7], t3 - t2);
    }
#endif
}

struct FrArgs {
    int B, N, iters;
    const float *planes;   // tile layout of k_depuncture / k_demap_planes
    double2 *le1;          // [B][N]: the last iteration's Le1 (global scratch)
    int32_t *bits;         // [B][2N]
    double *lfinal;        // [B][2N] or null
    int n_used;
    double2 *le2;          // LG: [B][N] Le2 planes (global scratch)
};

// DVBRCS2_Turbo.decode (:464-537) of one codeword per workgroup (grid = B).
// ord: [N] the positions in perm's image (ascending), then the others.
// LG: Le2 in global scratch (N > 805; see fr_lds).  WPD: waves per recursion
// direction (1: one wave, segments and rounds inside it, no cross-wave barriers;
// 2: fr_recursion_x), chosen per call by N (tdec_api.hip fr_wpd).
template <bool LG, int ALGO = 0, int WPD = FR_WPD_MAX>
__global__ __launch_bounds__(FR_BLOCK) void k_turbo_decode_frame(FrArgs p, const int *__restrict__ perm,
                                                                 const int *__restrict__ inv,
                                                                 const int *__restrict__ ord) {
    extern __shared__ float4 fr_sm[];
    lds_b *sm = (lds_b *)fr_sm;
    const int N = p.N, tid = threadIdx.x;
    const long cw = blockIdx.x;
    const FrLds Lo = fr_lds(N, true, LG);
    const long tile = cw / WAVE;
    const int cwl = (int)(cw % WAVE);
    const float *base = p.planes + tile * tile_floats(N);
    const float4 *X = reinterpret_cast<const float4 *>(base);
    const float2 *Z = reinterpret_cast<const float2 *>(base + (long)N * WAVE * 4);
    lds_int *sperm = (lds_int *)(sm + Lo.perm), *sinv = (lds_int *)(sm + Lo.inv);
    double2 *le2g = LG ? p.le2 + cw * N : nullptr;
    lds_d2 *le2s = (lds_d2 *)(sm + Lo.le2);
    // this thread's positions and their planes, once for all 16 SISOs
    int pos[FR_J];
    float4 xr[FR_J];
    float2 zr[FR_J];
#pragma unroll
    for (int j = 0; j < FR_J; ++j) {
        const int i = tid + j * FR_BLOCK;
        pos[j] = i < N ? ord[i] : -1;
        const int k = pos[j] < 0 ? 0 : pos[j];
        xr[j] = X[(long)k * WAVE + cwl];
        zr[j] = Z[(long)k * WAVE + cwl];
    }
    for (int k = tid; k < N; k += FR_BLOCK) {
        sperm[k] = perm[k];
        sinv[k] = inv[k];
        if constexpr (LG) le2g[k] = make_double2(0.0, 0.0);   // the first iteration's a-priori (:490-491)
        else le2s[k] = d2v{0.0, 0.0};
    }
    __syncthreads();   // (a workgroup barrier orders the workgroup's global accesses too: one CU, one L1)
    double2 *le1 = p.le1 + cw * N;
    for (int it = 0; it < p.iters; ++it) {
        const double sf = it < p.iters - 1 ? 0.7 : 1.0;   // :496
        const bool last = it == p.iters - 1;
        if constexpr (LG) {
            fr_siso<ALGO, WPD>(FrIn1T<const double2 *>{le2g, sinv}, FrOut1{sm + Lo.p1, last ? le1 : nullptr, p.n_used}, pos,
                          xr, sm, Lo, N, sf);
            fr_siso<ALGO, WPD>(FrIn2{sm + Lo.p1, sperm}, FrOut2T<double2 *>{le2g}, pos, zr, sm, Lo, N, sf);
        } else {
            fr_siso<ALGO, WPD>(FrIn1{le2s, sinv}, FrOut1{sm + Lo.p1, last ? le1 : nullptr, p.n_used}, pos, xr, sm, Lo, N, sf);
            fr_siso<ALGO, WPD>(FrIn2{sm + Lo.p1, sperm}, FrOut2T<lds_d2 *>{le2s}, pos, zr, sm, Lo, N, sf);
        }
    }
    // hard decision (:526-537): L = (Lc + La) + Le1, La = Le2[inv_perm]
#pragma unroll
    for (int j = 0; j < FR_J; ++j) {
        const int k = pos[j];
        if (k < 0) continue;
        const float4 x = xr[j];
        double lax, lay;
        if constexpr (LG) {
            const double2 la = le2g[sinv[k]];
            lax = la.x, lay = la.y;
        } else {
            const d2v la = le2s[sinv[k]];
            lax = la.x, lay = la.y;
        }
        const double2 le = le1[k];
        const double fa = ((double)x.x + lax) + le.x;
        const double fb = ((double)x.y + lay) + le.y;
        *reinterpret_cast<int2 *>(p.bits + cw * 2 * N + 2 * k) = make_int2(fa < 0.0 ? 1 : 0, fb < 0.0 ? 1 : 0);
        if (p.lfinal) *reinterpret_cast<double2 *>(p.lfinal + cw * 2 * N + 2 * k) = make_double2(fa, fb);
    }
}

// bcjr_max_log_map (:116-281) on [B][N] rows, one row per workgroup.
struct FrSisoArgs {
    int B, N;
    const void *LcA, *LcB, *LcW, *LcY;   // float32, or float64 for k_siso_frame<double>
    const double *LaA, *LaB;
    double sf;
    double *LeA, *LeB;
    unsigned *done;   // nullable: host-mapped per-row completion flags, set to seq after the row's outputs
    unsigned seq;
};
template <typename T, int ALGO = 0, int WPD = FR_WPD_MAX>
__global__ __launch_bounds__(FR_BLOCK) void k_siso_frame(FrSisoArgs p) {
    extern __shared__ float4 fr_sm[];
    lds_b *sm = (lds_b *)fr_sm;
    const long row = (long)blockIdx.x * p.N;
    const FrInRow<T> in{(const T *)p.LcA + row, (const T *)p.LcB + row, (const T *)p.LcW + row, (const T *)p.LcY + row,
                        p.LaA + row, p.LaB + row};
    int pos[FR_J];
    FrRowRaw<T> raw[FR_J];
#pragma unroll
    for (int j = 0; j < FR_J; ++j) {
        const int i = threadIdx.x + j * FR_BLOCK;
        pos[j] = i < p.N ? i : -1;
        raw[j] = in.fetch(i < p.N ? i : 0);
    }
    fr_siso<ALGO, WPD>(in, FrOutRow{p.LeA + row, p.LeB + row}, pos, raw, sm, fr_lds(p.N, false), p.N, p.sf);
    if (p.done) {
        // every thread's extrinsic stores are system-visible before the row's flag:
        // the host polls the flags instead of waiting for the kernel's end
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(p.done + blockIdx.x, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace tdec
