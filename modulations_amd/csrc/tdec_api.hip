// tdec_api.hip -- the C ABI (include/tdec.h) over the gfx950 kernels.
//
// Host-pointer entry points stage through handle-owned, grow-only device
// buffers and synchronise; _dev entry points are stream-ordered, allocation
// free once tdec_reserve() has sized the workspace (hipGraph-capturable).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "tdec.h"
#include "tdec_kernels.hip"
#include "tdec_workload.hip"
#include "tdec_spl.hip"
#include "tdec_lowlat.hip"
#include "tdec_frame.hip"

using namespace tdec;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? TDEC_ENOMEM : TDEC_EHIP,                  \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, bytes) != hipSuccess) return fail(TDEC_ENOMEM, "hipMalloc failed");
        cap = bytes;
        return 0;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Page-locked host staging for the small host-pointer calls (grown on demand).
// dev: the buffer's device address (zero-copy kernels read / write it directly),
// looked up once per allocation instead of per call.  flags: hipHostMalloc flags
// (hipHostMallocDefault; the SISO completion flags take coherent, mapped memory,
// which the host may poll while the kernel that writes it still runs).
struct PinBuf {
    void *p = nullptr, *dev = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes, unsigned flags = hipHostMallocDefault) {
        if (bytes <= cap) return 0;
        if (p) hipHostFree(p);
        p = dev = nullptr;
        cap = 0;
        if (hipHostMalloc(&p, bytes, flags) != hipSuccess) return fail(TDEC_ENOMEM, "hipHostMalloc failed");
        if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) dev = nullptr;
        cap = bytes;
        return 0;
    }
    void release() {
        if (p) hipHostFree(p);
        p = dev = nullptr;
        cap = 0;
    }
};

// A device buffer built from physical chunks mapped into one virtual range in a
// shuffled order (HIP virtual memory management): the physical placement of the
// decoder workspace is scattered BY CONSTRUCTION instead of by the placement
// probe's trial allocations (workspace placement).
struct VmmBuf {
    void *va = nullptr;
    size_t size = 0, chunk = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
    int alloc(int device, size_t bytes, size_t chunk_bytes, unsigned seed) {
        release();
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = device;
        size_t gran = 0;
        if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess || !gran)
            return fail(TDEC_EHIP, "hipMemGetAllocationGranularity failed");
        chunk = (std::max(chunk_bytes, gran) + gran - 1) / gran * gran;
        const size_t n = (bytes + chunk - 1) / chunk;
        size = n * chunk;
        if (hipMemAddressReserve(&va, size, 0, nullptr, 0) != hipSuccess) {
            va = nullptr;
            return fail(TDEC_ENOMEM, "hipMemAddressReserve failed");
        }
        h.resize(n);
        dev = device;
        std::vector<size_t> order(n);
        shuffled(order, seed);
        for (size_t i = 0; i < n; ++i) {
            if (hipMemCreate(&h[i], chunk, &prop, 0) != hipSuccess) {
                h.resize(i);
                release();
                return fail(TDEC_ENOMEM, "hipMemCreate failed (decoder workspace)");
            }
            if (hipMemMap((char *)va + order[i] * chunk, chunk, 0, h[i], 0) != hipSuccess) {
                h.resize(i + 1);
                release();
                return fail(TDEC_EHIP, "hipMemMap failed");
            }
        }
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        if (hipMemSetAccess(va, size, &acc, 1) != hipSuccess) {
            release();
            return fail(TDEC_EHIP, "hipMemSetAccess failed");
        }
        return 0;
    }
    static void shuffled(std::vector<size_t> &order, unsigned seed) {
        const size_t n = order.size();
        for (size_t i = 0; i < n; ++i) order[i] = i;
        unsigned long long x = 0x9E3779B97F4A7C15ull ^ seed;   // splitmix shuffle (deterministic)
        for (size_t i = n; i > 1; --i) {
            x += 0x9E3779B97F4A7C15ull;
            unsigned long long z = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            std::swap(order[i - 1], order[z % i]);
        }
    }
    int dev = 0;
    void release() {
        if (va && size) hipMemUnmap(va, size);
        for (auto &x : h) hipMemRelease(x);
        h.clear();
        if (va) hipMemAddressFree(va, size);
        va = nullptr;
        size = 0;
    }
};

struct Guard {  // select the handle's device for the duration of a call
    int prev = -1;
    explicit Guard(int dev) {
        hipGetDevice(&prev);
        if (prev != dev) hipSetDevice(dev);
    }
    ~Guard() {
        int cur;
        hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) hipSetDevice(prev);
    }
};

bool standard_trellis(const int32_t *t) {
    for (int s = 0; s < 16; ++s)
        for (int i = 0; i < 4; ++i) {
            if (t[0 * 64 + s * 4 + i] != t_next(s, i)) return false;
            if (t[1 * 64 + s * 4 + i] != t_ow(s, i)) return false;
            if (t[2 * 64 + s * 4 + i] != t_oy(s, i)) return false;
            if (t[3 * 64 + s * 4 + i] != t_prev_s(s, i)) return false;
            if (t[4 * 64 + s * 4 + i] != t_prev_i(s, i)) return false;
        }
    return true;
}

// GF(2) circular-state solve of the encoder (dvb_rcs2_turbo.py:37-114).
void mat_mul_gf2(const int *A, const int *B, int *C) {
    int T[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            int v = 0;
            for (int k = 0; k < 4; ++k) v ^= A[i * 4 + k] & B[k * 4 + j];
            T[i * 4 + j] = v;
        }
    std::memcpy(C, T, sizeof T);
}

int solve_circ(const int *Gp, int Z) {
    int M[4][5];
    for (int i = 0; i < 4; ++i) {
        for (int j = 0; j < 4; ++j) M[i][j] = ((i == j) + Gp[i * 4 + j]) % 2;
        M[i][4] = (Z >> i) & 1;
    }
    for (int i = 0; i < 4; ++i) {
        if (M[i][i] == 0)
            for (int k = i + 1; k < 4; ++k)
                if (M[k][i] == 1) {
                    for (int j = 0; j < 5; ++j) std::swap(M[i][j], M[k][j]);
                    break;
                }
        if (M[i][i] == 1)
            for (int k = i + 1; k < 4; ++k)
                if (M[k][i] == 1)
                    for (int j = 0; j < 5; ++j) M[k][j] ^= M[i][j];
    }
    int x[4] = {0, 0, 0, 0};
    for (int i = 3; i >= 0; --i) {
        int s = M[i][4];
        for (int j = i + 1; j < 4; ++j) s ^= M[i][j] & x[j];
        x[i] = s;
    }
    int st = 0;
    for (int i = 0; i < 4; ++i)
        if (x[i]) st |= 1 << i;
    return st;
}

// Constellation table to device memory, in the arithmetic dtype.  The upload
// synchronises once; later calls with the same table find it cached and stay
// fully stream-ordered.
// Device copy of a demapper table.  A table of M = 2^bps points (bps even,
// >= 4) whose point m is exactly levI[m >> bps/2] + j levQ[m & (2^(bps/2)-1)]
// is flagged separable and its axis levels are appended after the points.
struct ConsCache {
    DevBuf buf;
    std::vector<double> host;
    bool f64 = false;
    int sep = 0, nbps = -1;
    bool matches(const void *cons, int cons_f64, int M, int bps, bool want_f64) const {
        if (!buf.p || f64 != want_f64 || nbps != bps || (int)host.size() != 2 * M) return false;
        for (int i = 0; i < 2 * M; ++i)
            if (host[i] != (cons_f64 ? ((const double *)cons)[i] : (double)((const float *)cons)[i])) return false;
        return true;
    }
    int upload(const void *cons, int cons_f64, int M, int bps, bool want_f64, hipStream_t st) {
        std::vector<double> d(2 * M);
        for (int i = 0; i < 2 * M; ++i)
            d[i] = cons_f64 ? ((const double *)cons)[i] : (double)((const float *)cons)[i];
        if (buf.p && d == host && f64 == want_f64 && nbps == bps) return 0;
        if (int rc = buf.ensure(sizeof(double) * DM_TAB)) return rc;
        int s = bps >= 4 && bps % 2 == 0 && M == (1 << bps);
        const int K = bps / 2, L = 1 << K;
        std::vector<double> lev;
        if (s) {
            lev.resize(2 * L);
            for (int a = 0; a < L; ++a) lev[a] = d[2 * (a << K)];
            for (int q = 0; q < L; ++q) lev[L + q] = d[2 * q + 1];
            for (int m = 0; m < M && s; ++m)
                s = d[2 * m] == lev[m >> K] && d[2 * m + 1] == lev[L + (m & (L - 1))];
        }
        if (s) d.insert(d.end(), lev.begin(), lev.end());
        // Gray-labelled uniform PAM per axis (sym_llrs_gray): the level of label a sits
        // at position a ^ (a >> 1) of the ascending order, spacings equal within 1 %;
        // then the levels in position order and {x_0, 1/delta} per axis follow
        if (s) {
            std::vector<double> pos(2 * L), prm(4);
            for (int ax = 0; ax < 2 && s; ++ax) {
                const double *lv = lev.data() + ax * L;
                for (int a = 0; a < L; ++a) pos[ax * L + (a ^ (a >> 1))] = lv[a];
                for (int q = 0; q + 1 < L && s; ++q) s = pos[ax * L + q] < pos[ax * L + q + 1] ? s : 0;
                const double delta = (pos[ax * L + L - 1] - pos[ax * L]) / (L - 1);
                for (int q = 0; q + 1 < L && s; ++q)
                    s = std::fabs(pos[ax * L + q + 1] - pos[ax * L + q] - delta) <= 0.01 * delta ? s : 0;
                prm[2 * ax] = pos[ax * L];
                prm[2 * ax + 1] = 1.0 / delta;
            }
            if (s) {
                s = 2;
                d.insert(d.end(), pos.begin(), pos.end());
                d.insert(d.end(), prm.begin(), prm.end());
                // nb[b][p] = {nearest position left of p, right of p} whose label
                // (the inverse Gray code of the position) differs from p's in bit b
                // (MSB first); -1 / L when there is none
                auto lab = [&](int q) { int a = q; for (int sh = 1; sh < K; ++sh) a ^= q >> sh; return a; };
                for (int b = 0; b < K; ++b)
                    for (int q = 0; q < L; ++q) {
                        const int v = (lab(q) >> (K - 1 - b)) & 1;
                        int lq = q - 1, rq = q + 1;
                        while (lq >= 0 && ((lab(lq) >> (K - 1 - b)) & 1) == v) --lq;
                        while (rq < L && ((lab(rq) >> (K - 1 - b)) & 1) == v) ++rq;
                        d.push_back(lq);
                        d.push_back(rq);
                    }
            }
            else s = 1;
        }
        std::vector<float> f(d.begin(), d.end());   // exact: an f32 table only meets f32 arithmetic
        if (want_f64) HIPCHK(hipMemcpyAsync(buf.p, d.data(), sizeof(double) * d.size(), hipMemcpyHostToDevice, st));
        else HIPCHK(hipMemcpyAsync(buf.p, f.data(), sizeof(float) * f.size(), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        d.resize(2 * M);
        host = d;
        f64 = want_f64;
        sep = s;
        nbps = bps;
        return 0;
    }
};

// ---- demapper -------------------------------------------------------------------------
// compute_llr's configuration: noise_var floored at 0.005 (:202)
static DemapCfg demap_cfg(int M, int div_f32, int sign, double noise_var, int sep) {
    const double nv = (0.005 > noise_var) ? 0.005 : noise_var;
    return DemapCfg{M, div_f32, sign, nv, sep, dm_nv_fast(nv)};
}

template <typename T, typename S>
int launch_demap(int bps, const S *d_syms, long n_sym, const T *d_cons, DemapCfg c, double *d_llr,
                        hipStream_t st) {
    const dim3 grid((unsigned)((n_sym + BLOCK - 1) / BLOCK));
    switch (bps) {
#define CASE(K) \
    case K: hipLaunchKernelGGL((k_demap<T, S, K>), grid, dim3(BLOCK), 0, st, d_syms, n_sym, d_cons, c, d_llr); break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
    default: return fail(TDEC_EINVAL, "bps must be 1..8");
    }
    HIPCHK(hipGetLastError());
    return 0;
}

int check_demap_args(int M, int bps) {
    if (bps < 1 || bps > 8 || M < 1 || M > (1 << bps) || M > 256) return fail(TDEC_EINVAL, "bad constellation size");
    return 0;
}

typedef void (*decode_fn)(DecodeArgs, const int *, const int *, const int *);

const void *decode_kernel(int algo, bool ragged) {
    if (algo) return ragged ? (const void *)k_turbo_decode_logmap<true> : (const void *)k_turbo_decode_logmap<false>;
    return ragged ? (const void *)k_turbo_decode<true> : (const void *)k_turbo_decode<false>;
}

}  // namespace

constexpr size_t SIMD_PROG_BYTES = sizeof(int) * 8192 * 16;   // [XCC, SE, SH, CU, SIMD] key x 16 wave slots
struct tdec_ctx {
    int device = 0, N = 0, period = 1, iters = 8, algo = 0;
    uint8_t punct[16] = {0};
    long llr_len = 0, enc_len = 0;
    int circ[16] = {0};
    int max_waves = 0;                 // resident waves of the decode kernel on this device
    int n_cu = 0;                      // compute units of the device
    int32_t *d_perm = nullptr, *d_inv = nullptr, *d_src = nullptr, *d_off = nullptr;
    int32_t *d_dst = nullptr;          // LLR index -> c * N + k of the plane component it feeds (-1: none)
    // k_demap_planes' decline list (split tables): entries, count, per-tile overflow flags
    int2 *d_decl = nullptr;
    unsigned *d_decl_n = nullptr;
    unsigned char *d_decl_ovf = nullptr;
    long decl_tiles = 0;
    int32_t *d_used = nullptr;         // [N]: k in the image of perm
    int32_t *d_ulist = nullptr;        // [n_used]: the k in the image of perm, ascending (low-latency decoder)
    int32_t *d_ford = nullptr;         // [N]: those k, then the others (frame decoder's position order)
    int n_used = 0;
    int max_couple_llrs = 0;           // most LLRs any couple consumes (<= 6)
    DevBuf ws;                         // per-wave decode workspace: extrinsic planes + checkpoints
    VmmBuf ws_vmm;                     //   as shuffled physical chunks (>= 1 GiB)
    double2 *le_p = nullptr;           //   extrinsic planes P1 / Le2 / Le1 (inside ws)
    double2 *aux_p = nullptr;          //   a zero row (64 lanes) + per-wave sink rows (inside ws)
    int *d_tile_ctr = nullptr;         // the decoders' tile queue counter (zeroed before each launch)
    unsigned *d_tail = nullptr;        // the throughput decoder's tail flag (DecodeArgs::tail_flag)
    unsigned tail_seq = 0;             // sequence number of its last whole-tile launch
    int *d_simd_prog = nullptr;        // max-log issue priority: per-SIMD progress slots (zeroed before each launch)
    float4 *ck_p = nullptr;            //   alpha checkpoints + beta1 ring (inside ws)
    int ws_waves = 0;
    DevBuf planes_own;                 // planes for tdec_decode_batch(_dev)
    int cap_batch = 0;
    DevBuf h_llr, h_bits, h_lf, h_misc; // staging for the host-pointer API
    PinBuf pin;                        // page-locked staging of the small host-pointer calls
    PinBuf pin_siso;                   // the caller-filled SISO staging (tdec_siso_staging), never regrown behind its views
    PinBuf pin_flags;                  //   its per-row completion flags (fine-grained: coherent while a kernel runs)
    int siso_rows = 0;                 //   rows it holds
    unsigned siso_seq = 0;             //   the last call's sequence number in its completion flags
    long siso_fallbacks = 0;           //   staged calls that ended by a stream wait instead of their flags
    ConsCache cons;                    // demapper constellation
    DevBuf spl_ck;                     // checkpoints of the state-per-lane SISO prototype (TDEC_SISO_SPL=1)
    DevBuf planes_w;                   // per-wave plane buffers of the fused demap + decode
    DevBuf ll_ws, ll_st;               // small-batch decoders: extrinsic planes (frame: Le1 only), alpha / beta stores
    hipStream_t stream = nullptr;
    hipStream_t cstream = nullptr;     // uploads of the chunked host-pointer path (created on first use)
    hipStream_t dstream = nullptr;     // its downloads (a second copy engine direction)
    // Stream ordering of the handle-owned buffers (workspace, planes_own, cons,
    // staging): every call that touches them records done_ev on the stream it
    // ran on; a later call on a different stream waits on it first, so a
    // decode_device() on one stream followed by a decode_batch() (private
    // stream) or a _dev call on another stream cannot overwrite buffers a
    // running kernel still reads.
    hipEvent_t done_ev = nullptr;
    hipStream_t last_st = nullptr;
    bool pending = false;
};

namespace {
bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
// host-side wait for the last queued use (before buffers are regrown or staged)
void quiesce(tdec_ctx *h) {
    if (h->pending) hipEventSynchronize(h->done_ev);
}
// make stream s wait for the last use of the handle's buffers (on another stream)
int order_on(tdec_ctx *h, hipStream_t s) {
    if (h->pending && h->last_st != s && !capturing(s)) HIPCHK(hipStreamWaitEvent(s, h->done_ev, 0));
    return 0;
}
// the handle's buffers are in use by work queued on s
int mark_used(tdec_ctx *h, hipStream_t s) {
    if (capturing(s)) return 0;   // under stream capture the caller orders the graph
    HIPCHK(hipEventRecord(h->done_ev, s));
    h->last_st = s;
    h->pending = true;
    return 0;
}
// On every exit of a host-pointer entry point: the copies queued on the
// handle's streams read / write the caller's host buffers, so they must have
// finished before the caller gets control back (errors included).
struct DrainOnExit {
    hipStream_t a, b;
    ~DrainOnExit() {
        if (a) hipStreamSynchronize(a);
        if (b && b != a) hipStreamSynchronize(b);
    }
    void disarm() { a = b = nullptr; }   // the call synchronised its streams itself
};
// A host-pointer call that synchronised its stream leaves nothing queued on the
// handle's buffers: no event to record (mark_used) and none to wait on later.
void mark_idle(tdec_ctx *h) { h->pending = false; }
}  // namespace

extern "C" {

const char *tdec_last_error(void) { return g_err.c_str(); }

int tdec_create(int device, int n_couples, int period, const uint8_t *punct, int iterations, int algo,
                const int32_t *perm, const int32_t *inv_perm, const int32_t *tables, tdec_t **out) {
    if (!out || !punct || !perm || !inv_perm || !tables) return fail(TDEC_EINVAL, "null argument");
    *out = nullptr;
    if (n_couples <= 0) return fail(TDEC_EINVAL, "n_couples must be positive");
    if (period < 1 || period > 4) return fail(TDEC_EINVAL, "puncture period must be 1..4");
    if (iterations < 1) return fail(TDEC_EITER, "iterations must be >= 1");
    if (algo != TDEC_ALGO_MAXLOG && algo != TDEC_ALGO_LOGMAP) return fail(TDEC_EINVAL, "unknown algorithm");
    if (!standard_trellis(tables))
        return fail(TDEC_EUNSUPPORTED, "trellis tables are not the DVB-RCS2 16-state CRSC trellis");
    for (int k = 0; k < n_couples; ++k)
        if (perm[k] < 0 || perm[k] >= n_couples || inv_perm[k] < 0 || inv_perm[k] >= n_couples)
            return fail(TDEC_EINVAL, "perm / inv_perm entry out of range");
    int ndev = 0;
    const hipError_t dc = hipGetDeviceCount(&ndev);
    if (dc != hipSuccess || device < 0 || device >= ndev) {
        char msg[160];
        snprintf(msg, sizeof msg, "no such HIP device (device %d, hipGetDeviceCount: %d devices, %s)", device, ndev,
                 hipGetErrorString(dc));
        return fail(TDEC_EHIP, msg);
    }
    Guard g(device);
    auto *h = new tdec_ctx;
    h->device = device;
    h->N = n_couples;
    h->period = period;
    h->iters = iterations;
    h->algo = algo;
    std::memcpy(h->punct, punct, 16);
    const int N = n_couples;
    // de-puncture walk (:476-487) -> src[c*N + k] (LLR index or -1) for the 8 float4
    // components of the tile planes (X = A, B, W1, Y1; Z = -, -, W2, Y2)
    std::vector<int32_t> src(8 * (size_t)N, -1);
    long idx = 0;
    static const int comp_of_row[4] = {2, 3, 6, 7};   // W1 -> X.z, Y1 -> X.w, W2 -> Z.z, Y2 -> Z.w
    for (int i = 0; i < N; ++i) {
        const int p = i % period;
        src[0 * (size_t)N + i] = (int32_t)idx++;
        src[1 * (size_t)N + i] = (int32_t)idx++;
        for (int r = 0; r < 4; ++r) {
            if (punct[r * 4 + p]) src[comp_of_row[r] * (size_t)N + i] = (int32_t)idx++;
        }
    }
    h->llr_len = idx;
    h->enc_len = idx;   // encode() writes exactly what decode() reads (:449-460)
    std::vector<int32_t> off(N + 1);
    for (int i = 0; i < N; ++i) off[i] = src[i];      // A of couple i is its first LLR
    off[N] = (int32_t)idx;
    for (int i = 0; i < N; ++i) h->max_couple_llrs = std::max(h->max_couple_llrs, off[i + 1] - off[i]);
    if (h->max_couple_llrs > DM_MAXL / DM_KC) {   // the fused demapper's LDS tile assumes <= 6 LLRs per couple
        delete h;
        return fail(TDEC_EINVAL, "puncture pattern consumes more than 6 LLRs per couple");
    }
    // encoder circular-state table: S_c = solve((I + G^N), Z) for every Z (:414-417)
    int G[16] = {0};
    G[0 * 4 + 2] = G[0 * 4 + 3] = G[1 * 4 + 0] = G[2 * 4 + 1] = G[3 * 4 + 2] = 1;
    int res[16], base[16];
    for (int i = 0; i < 16; ++i) res[i] = (i % 5) == 0;
    std::memcpy(base, G, sizeof base);
    for (long pw = N; pw > 0; pw /= 2) {
        if (pw % 2 == 1) mat_mul_gf2(res, base, res);
        mat_mul_gf2(base, base, base);
    }
    for (int z = 0; z < 16; ++z) h->circ[z] = solve_circ(res, z);

    hipError_t e = hipSuccess;
    std::vector<int32_t> used(N, 0);
    for (int k = 0; k < N; ++k) used[perm[k]] = 1;
    e = hipMalloc(&h->d_perm, sizeof(int32_t) * N);
    if (e == hipSuccess) e = hipMalloc(&h->d_used, sizeof(int32_t) * N);
    if (e == hipSuccess) e = hipMemcpy(h->d_used, used.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice);
    std::vector<int32_t> ulist;
    for (int k = 0; k < N; ++k)
        if (used[k]) ulist.push_back(k);
    h->n_used = (int)ulist.size();
    if (e == hipSuccess) e = hipMalloc(&h->d_ulist, sizeof(int32_t) * N);
    if (e == hipSuccess) e = hipMemcpy(h->d_ulist, ulist.data(), sizeof(int32_t) * ulist.size(), hipMemcpyHostToDevice);
    std::vector<int32_t> ford(ulist);
    for (int k = 0; k < N; ++k)
        if (!used[k]) ford.push_back(k);
    if (e == hipSuccess) e = hipMalloc(&h->d_ford, sizeof(int32_t) * N);
    if (e == hipSuccess) e = hipMemcpy(h->d_ford, ford.data(), sizeof(int32_t) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&h->d_inv, sizeof(int32_t) * N);
    if (e == hipSuccess) e = hipMalloc(&h->d_src, sizeof(int32_t) * 8 * N);
    std::vector<int32_t> dst(std::max<long>(1, h->llr_len), -1);
    for (int cc = 0; cc < 8; ++cc)
        for (int k = 0; k < N; ++k)
            if (src[(size_t)cc * N + k] >= 0) dst[src[(size_t)cc * N + k]] = cc * N + k;
    if (e == hipSuccess) e = hipMalloc(&h->d_dst, sizeof(int32_t) * dst.size());
    if (e == hipSuccess) e = hipMemcpy(h->d_dst, dst.data(), sizeof(int32_t) * dst.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&h->d_tile_ctr, sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&h->d_tail, sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(h->d_tail, 0, sizeof(unsigned));
    if (e == hipSuccess && algo == TDEC_ALGO_MAXLOG) e = hipMalloc(&h->d_simd_prog, SIMD_PROG_BYTES);
    if (e == hipSuccess) e = hipMalloc(&h->d_off, sizeof(int32_t) * (N + 1));
    if (e == hipSuccess) e = hipMemcpy(h->d_off, off.data(), sizeof(int32_t) * (N + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->d_perm, perm, sizeof(int32_t) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->d_inv, inv_perm, sizeof(int32_t) * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->d_src, src.data(), sizeof(int32_t) * 8 * N, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->done_ev, hipEventDisableTiming);
    int blocks_per_cu = 0, n_cu = 0;
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &blocks_per_cu, decode_kernel(algo, n_couples % win_of(algo) != 0), DEC_BLOCK, 0);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) {
        tdec_destroy(h);
        return fail(TDEC_EHIP, std::string("tdec_create: ") + hipGetErrorString(e));
    }
    h->max_waves = std::max(1, blocks_per_cu) * n_cu * DEC_WAVES;
    h->n_cu = n_cu;
    // the kernels address one workspace plane / the checkpoint array with 32-bit
    // byte offsets: rows of n_waves * 64 lanes must keep them below 4 GiB
    const long row_units = std::max<long>(rows_of(N), 4L * ((N + ck_win_of(algo) - 1) / ck_win_of(algo) + RING));
    const long cap = (long)(4294967295UL / ((unsigned long)row_units * WAVE * 16UL));
    h->max_waves = (int)std::max<long>(1, std::min<long>(h->max_waves, cap));
    *out = h;
    return TDEC_OK;
}

void tdec_destroy(tdec_t *h) {
    if (!h) return;
    Guard g(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    if (h->pending) hipEventSynchronize(h->done_ev);
#if TDEC_PASS_TIMING
    {   // measurement build: per-pass cycles of every decode since the last destroy
        unsigned long long c[8] = {};
        hipDeviceSynchronize();
        if (hipMemcpyFromSymbol(c, HIP_SYMBOL(g_pass_cycles), sizeof(c)) == hipSuccess) {
            const double t = (double)(c[0] + c[1] + c[2] + c[3] + c[4]);
            fprintf(stderr, "[tdec] pass cycles: F1 %.3f F2 %.3f B1 %.3f B2 %.3f epilogue %.3f (total %.3e)\n",
                    c[0] / t, c[1] / t, c[2] / t, c[3] / t, c[4] / t, t);
            const unsigned long long z[8] = {};
            hipMemcpyToSymbol(HIP_SYMBOL(g_pass_cycles), z, sizeof(z));
        }
        static unsigned long long mh[4][MH_END + 1];
        if (hipMemcpyFromSymbol(mh, HIP_SYMBOL(g_merge_hist), sizeof(mh)) == hipSuccess) {
            // merge depth in steps: bucket i = i * 8 steps; "end" = never merged
            static const char *name[4] = {"F2 lane", "F2 wave", "B2 lane", "B2 wave"};
            for (int w = 0; w < 4; ++w) {
                unsigned long long tot = 0, acc = 0;
                double mean = 0;
                for (int i = 0; i <= MH_END; ++i) tot += mh[w][i], mean += i < MH_END ? (double)i * 8 * mh[w][i] : 0;
                if (!tot) continue;
                fprintf(stderr, "[tdec] merge %s: n %llu mean(merged) %.1f steps", name[w], tot,
                        mean / std::max(1ull, tot - mh[w][MH_END]));
                const double q[5] = {0.5, 0.9, 0.99, 0.999, 1.0};
                int qi = 0;
                for (int i = 0; i <= MH_END && qi < 5; ++i) {
                    acc += mh[w][i];
                    while (qi < 5 && acc >= q[qi] * tot) fprintf(stderr, " p%g %d", q[qi++] * 100, i * 8);
                }
                fprintf(stderr, " end %.5f\n", (double)mh[w][MH_END] / tot);
            }
            memset(mh, 0, sizeof(mh));
            hipMemcpyToSymbol(HIP_SYMBOL(g_merge_hist), mh, sizeof(mh));
        }
    }
#endif
#if TDEC_WAVE_TIMING
    {   // measurement build: wave finish-time spread of the last decode launch
        static unsigned long long t[WT_MAX][4];
        static int nt[WT_MAX];
        hipDeviceSynchronize();
        const int n = std::min(h->max_waves, WT_MAX);
        if (n > 0 && hipMemcpyFromSymbol(t, HIP_SYMBOL(g_wave_t), sizeof(t)) == hipSuccess &&
            hipMemcpyFromSymbol(nt, HIP_SYMBOL(g_wave_tiles), sizeof(nt)) == hipSuccess) {
            unsigned long long t0 = ~0ull, t1 = 0;
            for (int i = 0; i < n; ++i) t0 = std::min(t0, t[i][0]), t1 = std::max(t1, t[i][1]);
            std::vector<double> end(n);
            double busy = 0;
            int tmin = 1 << 30, tmax = 0;
            for (int i = 0; i < n; ++i) {
                end[i] = (t[i][1] - t0) * 1e-5;   // ms at 100 MHz
                busy += (t[i][1] - t[i][0]) * 1e-5;
                tmin = std::min(tmin, nt[i]), tmax = std::max(tmax, nt[i]);
            }
            if (const char *dump = getenv("TDEC_WAVE_DUMP")) {   // per wave: start, end (ms), tiles, hw ids
                static unsigned hw[WT_MAX][2];
                if (FILE *f = fopen(dump, "a"); f && hipMemcpyFromSymbol(hw, HIP_SYMBOL(g_wave_hw), sizeof(hw)) == hipSuccess) {
                    fprintf(f, "# launch waves=%d\n", n);
                    for (int i = 0; i < n; ++i)
                        fprintf(f, "%d %llu %llu %d %u %u %llu %llu\n", i, t[i][0], t[i][1], nt[i], hw[i][0], hw[i][1],
                                t[i][2], t[i][3]);
                    fclose(f);
                }
            }
            // the shader clock each wave ran at: s_memtime ticks over s_memrealtime (100 MHz)
            double ck_sum = 0, ck_min = 1e30, ck_max = 0;
            for (int i = 0; i < n; ++i) {
                const double ghz = (double)(t[i][3] - t[i][2]) / std::max(1.0, (double)(t[i][1] - t[i][0]) * 10.0);
                ck_sum += ghz, ck_min = std::min(ck_min, ghz), ck_max = std::max(ck_max, ghz);
            }
            fprintf(stderr, "[tdec] wave clock: mean %.3f GHz (min %.3f, max %.3f)\n", ck_sum / n, ck_min, ck_max);
            std::sort(end.begin(), end.end());
            const double span = (t1 - t0) * 1e-5;
            fprintf(stderr,
                    "[tdec] waves %d: span %.2f ms, wave end p0 %.2f p10 %.2f p50 %.2f p90 %.2f p100 %.2f ms, "
                    "busy %.4f of waves x span, tiles per wave %d..%d\n",
                    n, span, end[0], end[n / 10], end[n / 2], end[n * 9 / 10], end[n - 1], busy / (n * span), tmin,
                    tmax);
            // mean tiles per wave by XCD (blocks are dispatched round-robin over the 8 XCDs), by
            // wave within the block and by the block's slot on its CU (block / 8 even or odd)
            double x[8] = {}, wb[4] = {}, sl[2] = {};
            int nx[8] = {}, nwb[4] = {}, nsl[2] = {};
            for (int i = 0; i < n; ++i) {
                const int blk = i / 4;
                x[blk % 8] += nt[i], ++nx[blk % 8];
                wb[i % 4] += nt[i], ++nwb[i % 4];
                sl[(blk / 8) & 1] += nt[i], ++nsl[(blk / 8) & 1];
            }
            fprintf(stderr, "[tdec] tiles/wave by XCD:");
            for (int i = 0; i < 8; ++i) fprintf(stderr, " %.2f", nx[i] ? x[i] / nx[i] : 0.0);
            fprintf(stderr, "  by wave in block:");
            for (int i = 0; i < 4; ++i) fprintf(stderr, " %.2f", nwb[i] ? wb[i] / nwb[i] : 0.0);
            fprintf(stderr, "  by block/8 parity: %.2f %.2f\n", nsl[0] ? sl[0] / nsl[0] : 0.0,
                    nsl[1] ? sl[1] / nsl[1] : 0.0);
            int hist[16] = {};
            for (int i = 0; i < n; ++i) ++hist[std::min(nt[i], 15)];
            fprintf(stderr, "[tdec] tiles/wave histogram:");
            for (int i = 0; i < 16; ++i)
                if (hist[i]) fprintf(stderr, " %d:%d", i, hist[i]);
            fprintf(stderr, "\n");
        }
    }
#endif
    hipFree(h->d_perm);
    hipFree(h->d_used);
    hipFree(h->d_ulist);
    hipFree(h->d_ford);
    hipFree(h->d_inv);
    hipFree(h->d_src);
    hipFree(h->d_dst);
    hipFree(h->d_decl);
    hipFree(h->d_decl_n);
    hipFree(h->d_decl_ovf);
    hipFree(h->d_tile_ctr);
    hipFree(h->d_tail);
    if (h->d_simd_prog) hipFree(h->d_simd_prog);
    hipFree(h->d_off);
    if (h->ws_vmm.va) h->ws.p = nullptr;   // the VMM range is not a hipMalloc pointer
    h->ws.release();
    h->ws_vmm.release();
    h->planes_own.release();
    h->h_llr.release();
    h->h_bits.release();
    h->h_lf.release();
    h->h_misc.release();
    h->pin.release();
    h->pin_siso.release();
    h->pin_flags.release();
    h->cons.buf.release();
    h->spl_ck.release();
    h->planes_w.release();
    h->ll_ws.release();
    h->ll_st.release();
    if (h->stream) hipStreamDestroy(h->stream);
    if (h->cstream) hipStreamDestroy(h->cstream);
    if (h->dstream) hipStreamDestroy(h->dstream);
    if (h->done_ev) hipEventDestroy(h->done_ev);
    delete h;
}

long tdec_llr_len(const tdec_t *h) { return h ? h->llr_len : TDEC_EINVAL; }

long tdec_encode_host(int n_couples, int period, const uint8_t *punct, const int32_t *perm, long B,
                      const int32_t *bits, long bits_stride, int32_t *out, long out_stride) {
    const int N = n_couples;
    if (N <= 0 || period < 1 || period > 4 || !punct || !perm || B < 0 || (B > 0 && (!bits || !out)))
        return fail(TDEC_EINVAL, "bad encode arguments");
    long n_out = 0;
    for (int i = 0; i < N; ++i) {
        n_out += 2;
        for (int r = 0; r < 4; ++r) n_out += punct[r * 4 + i % period] ? 1 : 0;
    }
    if (B > 0 && (bits_stride < 2L * N || out_stride < n_out)) return fail(TDEC_EINVAL, "encode row strides too short");
    for (int k = 0; k < N; ++k)
        if (perm[k] < 0 || perm[k] >= N) return fail(TDEC_EINVAL, "perm entry out of range");
    // circular-state table S_c = solve((I + G^N), Z) (:414-417), as tdec_create
    int G[16] = {0};
    G[0 * 4 + 2] = G[0 * 4 + 3] = G[1 * 4 + 0] = G[2 * 4 + 1] = G[3 * 4 + 2] = 1;
    int res[16], base[16], circ[16];
    for (int i = 0; i < 16; ++i) res[i] = (i % 5) == 0;
    std::memcpy(base, G, sizeof base);
    for (long pw = N; pw > 0; pw /= 2) {
        if (pw % 2 == 1) mat_mul_gf2(res, base, res);
        mat_mul_gf2(base, base, base);
    }
    for (int z = 0; z < 16; ++z) circ[z] = solve_circ(res, z);
    std::vector<int> in1(N), in2(N);
    std::vector<uint8_t> w1(N), y1(N), w2(N), y2(N);
    // one RSC component (:404-429): zero-state pass, circular start, encode pass
    auto component = [&](const std::vector<int> &in, std::vector<uint8_t> &W, std::vector<uint8_t> &Y) {
        int s = 0;
        for (int i = 0; i < N; ++i) s = t_next(s, in[i]);
        s = circ[s];
        for (int i = 0; i < N; ++i) {
            W[i] = (uint8_t)t_ow(s, in[i]);
            Y[i] = (uint8_t)t_oy(s, in[i]);
            s = t_next(s, in[i]);
        }
    };
    for (long b = 0; b < B; ++b) {
        const int32_t *x = bits + b * bits_stride;
        for (int i = 0; i < N; ++i) {
            // (A << 1) | B indexes next_state[state, :]: numpy wraps -4..-1, raises otherwise
            const int32_t v = (int32_t)((uint32_t)x[2 * i] << 1) | x[2 * i + 1];
            if (v < -4 || v > 3) return fail(TDEC_ESHORT, "index out of bounds for the next_state lookup (info bits must be 0/1)");
            in1[i] = v & 3;
        }
        for (int i = 0; i < N; ++i) {   // A[perm], B[perm] (:447-449)
            const int32_t *q = x + 2 * perm[i];
            in2[i] = (int)(((int32_t)((uint32_t)q[0] << 1) | q[1]) & 3);
        }
        component(in1, w1, y1);
        component(in2, w2, y2);
        int32_t *o = out + b * out_stride;
        long j = 0;
        for (int i = 0; i < N; ++i) {   // puncture / multiplex (:451-460)
            const int p = i % period;
            o[j++] = x[2 * i];
            o[j++] = x[2 * i + 1];
            if (punct[0 * 4 + p]) o[j++] = w1[i];
            if (punct[1 * 4 + p]) o[j++] = y1[i];
            if (punct[2 * 4 + p]) o[j++] = w2[i];
            if (punct[3 * 4 + p]) o[j++] = y2[i];
        }
    }
    return n_out;
}
long tdec_encoded_len(const tdec_t *h) { return h ? h->enc_len : TDEC_EINVAL; }

size_t tdec_planes_bytes(const tdec_t *h, int B) {
    if (!h || B <= 0) return 0;
    const size_t tiles = ((size_t)B + WAVE - 1) / WAVE;
    return tiles * (size_t)tile_floats(h->N) * sizeof(float);
}

static int n_tiles_of(int B) { return (B + WAVE - 1) / WAVE; }

// Per-wave workspace strides (elements).
static long ws_stride_of(const tdec_t *h) { return 3L * rows_of(h->N) * WAVE; }
static int ck_rows_of(const tdec_t *h) { return (h->N + ck_win_of(h->algo) - 1) / ck_win_of(h->algo); }
static long ck_stride_of(const tdec_t *h) { return (long)(ck_rows_of(h) + RING) * 4 * WAVE; }

// The decoders' tile queue: the counter zeroed on the launch's stream, or null
// (static striding) below 4 tiles per wave.  Measured (same bits): 1 M codewords
// (8 tiles per wave) 243.8 -> 241.6 ms; at 2 tiles per wave the queue was no
// faster (max-log 61.8 vs 62.6, log-MAP 381.2 vs 385.9 ms per 262 144), hence the
// threshold.
static int *tile_queue(tdec_t *h, int tiles, int waves, hipStream_t st) {
    if (tiles < 4 * waves) return nullptr;
    if (hipMemsetAsync(h->d_tile_ctr, 0, sizeof(int), st) != hipSuccess) return nullptr;
    return h->d_tile_ctr;
}

// Workspace for `waves` concurrently decoding waves: the extrinsic planes and
// the checkpoints in one allocation (checkpoints on the next 2 MiB boundary).
//
// Placement.  The decode rate depends on where in HBM this workspace lands: on
// MI355X a full-size workspace (6.4 GB at N = 752) from one hipMalloc decodes
// anywhere from ~70 to ~80 ms per 262 144 codewords depending on the physical
// pages it gets (DRAM read-credit stalls on a slow placement; the
// planes' placement does not matter).  A workspace of >= 1 GiB is therefore built
// from 64 MiB physical chunks mapped into one virtual range in a fixed shuffled
// order (VmmBuf), which places it scattered by construction: measured as fast as
// the best of a timed 8-16-candidate placement probe in every fresh process, with
// no transient trial allocations (profiles/r03m/, r03n/vmm_ab.txt; the probe,
// physically contiguous ranges, row padding, chunk sizes >= 128 MiB and searches
// over chunk orders are in the DESIGN.md appendix).  Smaller workspaces, or a
// device without VMM support, take one hipMalloc.
static int ensure_ws(tdec_t *h, int waves) {
    if (waves <= h->ws_waves) return 0;
    if (h->ws_vmm.va) {   // regrowth of a VMM workspace: drop it first (not a hipMalloc pointer)
        h->ws.p = nullptr;
        h->ws.cap = 0;
        h->ws_vmm.release();
    }
    const size_t MB2 = 2u << 20;
    // rows of waves*64 lanes: the planes have 3N rows, the checkpoints ck_stride_of / 64
    const size_t row = (size_t)waves * WAVE;
    const size_t le_bytes = row * (ws_stride_of(h) / WAVE) * sizeof(double2);
    const size_t ck_off = (le_bytes + MB2 - 1) / MB2 * MB2;
    // aux: the all-zero a-priori row of the first iteration (64 lanes, zeroed
    // below) and one sink row per wave for the stores the decoder discards
    const size_t aux_off = ck_off + row * (ck_stride_of(h) / WAVE) * sizeof(float4);
    const size_t total = aux_off + ((size_t)WAVE + row) * sizeof(double2);
    bool placed = false;
    if (total >= (1ul << 30)) {
        h->ws.release();
        if (h->ws_vmm.alloc(h->device, total, 64ul << 20, 12345u) == 0) {
            h->ws.p = h->ws_vmm.va;   // not owned by ws (released through ws_vmm)
            h->ws.cap = total;
            placed = true;
        } else {
            hipGetLastError();   // no VMM support: one hipMalloc below
        }
    }
    if (!placed)
        if (int rc = h->ws.ensure(total)) return rc;
    h->le_p = (double2 *)h->ws.p;
    h->ck_p = (float4 *)((char *)h->ws.p + ck_off);
    h->aux_p = (double2 *)((char *)h->ws.p + aux_off);
    HIPCHK(hipMemsetAsync(h->aux_p, 0, WAVE * sizeof(double2), h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    h->ws_waves = waves;
    return 0;
}

// Batches of at most lowlat_max() codewords (max-log) run the one-codeword-per-
// wave decoder (tdec_lowlat.hip): lower latency per call.  Measured (N=752 r=1/2,
// host-pointer call, profiles/r03h_latency.jsonl, r03i_latency_lowlat4096.json):
// B = 1 5.0 vs 11.1 ms, 256 6.7 vs 13.2 ms, 1024 9.0 vs 13.6 ms for the per-lane
// decoder.  TDEC_LOWLAT_MAX overrides the threshold (0 disables it).
// Round 4, the frame decoder against the throughput decoder (host-pointer calls,
// profiles/r04u/): N = 752 r = 1/2 B = 8 192 16.3 vs 19.7 ms, 16 384 32.9 vs 26.7 ms;
// N = 212 B = 4 096 4.3 vs 5.6 ms, 8 192 8.5 vs 6.2 ms: the threshold was 8 192 for
// N >= 400 and 4 096 below (round 5: 12 288 / 8 192, below).
static size_t ll_lds_bytes(int N) { return 3 * sizeof(int) * (size_t)N; }   // perm, inv_perm, used list
// The frame decoder (tdec_frame.hip, one codeword per workgroup, everything in
// LDS) takes the small batches when its LDS fits (N <= 805: every BASELINE
// config); the round-3 state-per-lane decoder (tdec_lowlat.hip) otherwise, or
// with TDEC_FRAME=0 (A/B).
// The decoder keeps Le2 in global scratch where its full LDS plan does not fit (N > 805).
static bool frame_le2_global(int N) { return fr_lds(N, true, false).total > FR_LDS_MAX; }
static bool frame_fits(int N, bool dec) {
    return N <= FR_J * FR_BLOCK && fr_lds(N, dec, dec && frame_le2_global(N)).total <= FR_LDS_MAX;
}
static bool use_frame_decoder(const tdec_t *h) {
    const char *e = getenv("TDEC_FRAME");   // read per call: tests switch decoders in-process
    return !(e && e[0] == '0') && frame_fits(h->N, true);
}
// log-MAP batches the frame decoder takes (TDEC_LOWLAT_MAX overrides it too).  Measured
// (profiles/r05/logmap_frame/, N = 752 r = 1/2, host-pointer calls): frame decoder
// 1.08 / 1.32 / 5.30 / 20.4 / 43.1 ms at B = 1 / 64 / 1 024 / 4 096 / 8 192, the
// throughput kernel 27.9 / 28.0 / 28.7 / 30.0 / 34.4 ms: the crossover is near 6 000.
// After the 8-step log-MAP frame blocks (profiles/r05/crossover_lm/): N = 752 r = 1/2
// frame 28.4 / 37.0 ms at B = 6 144 / 8 192 against 33.3 / 34.5, N = 212 7.9 / 10.6
// against 9.6 / 9.7: near 7 000 for both.
constexpr int LM_FRAME_MAX = 7168;
static int lowlat_max(const tdec_t *h) {
    static const int v = [] {
        const char *e = getenv("TDEC_LOWLAT_MAX");
        return e ? std::max(0, atoi(e)) : -1;
    }();
    if (h->algo != TDEC_ALGO_MAXLOG) {   // log-MAP: the frame decoder only (the state-per-lane one is max-log)
        if (!use_frame_decoder(h)) return 0;
        return v >= 0 ? v : LM_FRAME_MAX;
    }
    if (v >= 0) return v;
    // the state-per-lane decoder's own crossover is 4 096 (26.1 vs 20.2 ms at 8 192,
    // profiles/r03llmax/).  The frame decoder's, re-measured after round 5's frame
    // speedups (profiles/r05/crossover/, host-pointer decode_batch, frame vs
    // throughput decoder): N = 752 B = 8 192 13.5 vs 18.6 ms, 12 288 19.7 vs 22.7,
    // 16 384 26.3 vs 26.1; N = 212 B = 8 192 5.7 vs 6.1 ms, 12 288 8.4 vs 6.7
    if (!use_frame_decoder(h)) return 4096;
    return h->N >= 400 ? 12288 : 8192;
}
// One predicate for "the small-batch decoders can run on this handle" (reserve and decode).
static bool lowlat_usable(const tdec_t *h) {
    return lowlat_max(h) > 0 &&
           (use_frame_decoder(h) || (h->algo == TDEC_ALGO_MAXLOG && ll_lds_bytes(h->N) <= 64 * 1024));
}
// Codewords the small-batch workspace holds for the decoder that would run (batches
// up to that minus 4): the frame decoder keeps only Le1 (N double2 per row) outside
// LDS, the state-per-lane decoder three extrinsic planes and the alpha / beta stores.
static int ll_cap_of(const tdec_t *h) {
    if (use_frame_decoder(h))   // Le1 (and with Le2 in global scratch, Le2) per row
        return (int)std::min<size_t>(h->ll_ws.cap / ((frame_le2_global(h->N) ? 2 : 1) * (size_t)h->N * sizeof(double2)),
                                     1 << 30);
    return (int)std::min(h->ll_ws.cap / (ll_ws_elems(h->N) * sizeof(double2)), h->ll_st.cap / (ll_st_elems(h->N) * sizeof(float)));
}
static bool use_lowlat(const tdec_t *h, int B) {
    return B <= lowlat_max(h) && B + 4 <= ll_cap_of(h) && lowlat_usable(h);
}
// kernels with more than 64 KiB of dynamic LDS must say so, once per device (the
// attribute belongs to the kernel on the device current when it is set)
static int frame_lds_attr(int device) {
    static std::mutex mu;
    static unsigned char done[256];
    if (device < 0 || device >= 256) return fail(TDEC_EINVAL, "device ordinal out of range");
    std::lock_guard<std::mutex> lk(mu);
    if (done[device]) return 0;
    const void *fns[] = {(const void *)k_turbo_decode_frame<false, 0, 1>, (const void *)k_turbo_decode_frame<true, 0, 1>,
                         (const void *)k_turbo_decode_frame<false, 1, 1>, (const void *)k_turbo_decode_frame<true, 1, 1>,
                         (const void *)k_siso_frame<float, 0, 1>, (const void *)k_siso_frame<double, 0, 1>,
                         (const void *)k_siso_frame<float, 1, 1>, (const void *)k_siso_frame<double, 1, 1>,
                         (const void *)k_turbo_decode_frame<false, 0, 2>, (const void *)k_turbo_decode_frame<true, 0, 2>,
                         (const void *)k_turbo_decode_frame<false, 1, 2>, (const void *)k_turbo_decode_frame<true, 1, 2>,
                         (const void *)k_siso_frame<float, 0, 2>, (const void *)k_siso_frame<double, 0, 2>,
                         (const void *)k_siso_frame<float, 1, 2>, (const void *)k_siso_frame<double, 1, 2>};
    for (const void *f : fns) {
        const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, FR_LDS_MAX);
        if (r != hipSuccess) return fail(TDEC_EHIP, std::string("hipFuncSetAttribute (frame decoder LDS): ") + hipGetErrorString(r));
    }
    done[device] = 1;
    return 0;
}

// Waves per recursion direction of the frame kernels, by block length: one wave
// (segments and rounds inside it, no cross-wave barriers) up to fr_wpd1_max, two
// above (8 segments: shorter chains once N is long).  Measured (profiles/r05/wpd/):
// decode() per frame N = 48 0.132 -> 0.118 ms, 212 0.189 -> 0.149, 752 0.200 ->
// 0.248 (worse); one SISO call 0.024 -> 0.021, 0.037 -> 0.029, 0.038 -> 0.035.
// TDEC_FR_WPD1_MAX / TDEC_FR_SISO_WPD1_MAX override the limits (read per call).
static int fr_wpd(int N, bool siso) {
    const char *e = getenv(siso ? "TDEC_FR_SISO_WPD1_MAX" : "TDEC_FR_WPD1_MAX");
    const int lim = e ? atoi(e) : (siso ? 1 << 30 : 424);
    return N <= lim ? 1 : 2;
}

static int ensure_lowlat(tdec_t *h, int B) {
    if (B > lowlat_max(h) || B + 4 <= ll_cap_of(h) || !lowlat_usable(h)) return 0;
    const size_t cap = std::min(lowlat_max(h), std::max(B, 64)) + 4;
    if (use_frame_decoder(h)) return h->ll_ws.ensure(cap * (frame_le2_global(h->N) ? 2 : 1) * h->N * sizeof(double2));
    if (int rc = h->ll_ws.ensure(cap * ll_ws_elems(h->N) * sizeof(double2))) return rc;
    return h->ll_st.ensure(cap * ll_st_elems(h->N) * sizeof(float));
}

// k_demap_planes' decline list (entries + count, allocated once) and its per-tile
// overflow flags (grown with the batch).  The caller has quiesced the handle.
static int ensure_decl(tdec_t *h, long n_tiles) {
    if (!h->d_decl) {
        HIPCHK(hipMalloc(&h->d_decl, sizeof(int2) * DM_DECL_CAP));
        HIPCHK(hipMalloc(&h->d_decl_n, sizeof(unsigned)));
    }
    if (h->decl_tiles < n_tiles) {
        hipFree(h->d_decl_ovf);
        h->d_decl_ovf = nullptr;
        h->decl_tiles = 0;
        HIPCHK(hipMalloc(&h->d_decl_ovf, (size_t)n_tiles));
        h->decl_tiles = n_tiles;
    }
    return 0;
}

int tdec_reserve(tdec_t *h, int max_batch) {
    if (!h || max_batch < 0) return fail(TDEC_EINVAL, "bad reserve");
    if (max_batch == 0) return 0;
    Guard g(h->device);
    if (max_batch <= lowlat_max(h) && lowlat_usable(h)) {   // small batches: the frame / state-per-lane decoders' workspace only
        if (max_batch + 4 > ll_cap_of(h) || tdec_planes_bytes(h, max_batch) > h->planes_own.cap) quiesce(h);
        if (n_tiles_of(max_batch) > h->decl_tiles) quiesce(h);
        int rc = ensure_lowlat(h, max_batch);
        if (!rc) rc = h->planes_own.ensure(tdec_planes_bytes(h, max_batch));
        if (!rc) rc = ensure_decl(h, n_tiles_of(max_batch));   // the demapper's, for tdec_demap_planes_dev
        if (!rc) h->cap_batch = std::max(h->cap_batch, max_batch);
        return rc;
    }
    const int want_waves = std::min(n_tiles_of(max_batch), h->max_waves);
    if (want_waves > h->ws_waves || tdec_planes_bytes(h, max_batch) > h->planes_own.cap ||
        n_tiles_of(max_batch) > h->decl_tiles)
        quiesce(h);   // regrowth frees
    int rc = ensure_ws(h, want_waves);
    if (!rc) rc = h->planes_own.ensure(tdec_planes_bytes(h, max_batch));
    if (!rc) rc = ensure_decl(h, n_tiles_of(max_batch));
    if (!rc) h->cap_batch = std::max(h->cap_batch, max_batch);
    return rc;
}

int tdec_depuncture_dev(tdec_t *h, int B, const float *d_llr, long llr_stride, float *d_planes, void *stream) {
    if (!h || B < 0) return fail(TDEC_EINVAL, "bad depuncture arguments");
    if (B == 0) return 0;   // an empty batch is a no-op (every batched entry point)
    if (!d_llr || !d_planes) return fail(TDEC_EINVAL, "bad depuncture arguments");
    if (llr_stride < h->llr_len) return fail(TDEC_ESHORT, "llr rows shorter than the de-puncture walk");
    Guard g(h->device);
    const long total = (long)n_tiles_of(B) * h->N * WAVE;
    hipLaunchKernelGGL(k_depuncture, dim3((unsigned)((total + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                       (hipStream_t)stream, B, h->N, d_llr, llr_stride, (const int *)h->d_src, d_planes, total);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdec_decode_planes_dev(tdec_t *h, int B, const float *d_planes, int32_t *d_bits, double *d_lfinal,
                           void *stream) {
    if (!h || B < 0) return fail(TDEC_EINVAL, "bad decode arguments");
    if (B == 0) return 0;
    if (!d_planes || !d_bits) return fail(TDEC_EINVAL, "bad decode arguments");
    Guard g(h->device);
    hipStream_t st = (hipStream_t)stream;
    if (use_lowlat(h, B)) {
        if (int rc = order_on(h, st)) return rc;
        if (use_frame_decoder(h)) {
            if (int rc = frame_lds_attr(h->device)) return rc;
            const bool lg = frame_le2_global(h->N);
            FrArgs a{B, h->N, h->iters, d_planes, (double2 *)h->ll_ws.p, d_bits, d_lfinal, h->n_used,
                     lg ? (double2 *)h->ll_ws.p + (size_t)B * h->N : nullptr};
            const bool w1 = fr_wpd(h->N, false) == 1;
            const auto kern = h->algo ? (lg ? (w1 ? k_turbo_decode_frame<true, 1, 1> : k_turbo_decode_frame<true, 1, 2>)
                                            : (w1 ? k_turbo_decode_frame<false, 1, 1> : k_turbo_decode_frame<false, 1, 2>))
                                      : (lg ? (w1 ? k_turbo_decode_frame<true, 0, 1> : k_turbo_decode_frame<true, 0, 2>)
                                            : (w1 ? k_turbo_decode_frame<false, 0, 1> : k_turbo_decode_frame<false, 0, 2>));
            hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(FR_BLOCK), fr_lds(h->N, true, lg).total, st, a,
                               (const int *)h->d_perm, (const int *)h->d_inv, (const int *)h->d_ford);
            HIPCHK(hipGetLastError());
            return mark_used(h, st);
        }
        LLArgs a{B, h->N, h->iters, d_planes, (double2 *)h->ll_ws.p, (float *)h->ll_st.p, d_bits, d_lfinal,
                 (const int *)h->d_ulist, h->n_used};
        hipLaunchKernelGGL(k_turbo_decode_lowlat, dim3((unsigned)B), dim3(WAVE), ll_lds_bytes(h->N), st, a,
                           (const int *)h->d_perm, (const int *)h->d_inv);
        HIPCHK(hipGetLastError());
        return mark_used(h, st);
    }
    const int tiles = n_tiles_of(B);
    const int waves = std::min(tiles, h->max_waves);
    if (waves > h->ws_waves) return fail(TDEC_ECAPACITY, "workspace too small: call tdec_reserve first");
    if (int rc = order_on(h, st)) return rc;
    DecodeArgs a{B, h->N, h->iters, tiles, waves, d_planes, h->le_p, h->ck_p, d_bits, d_lfinal, h->d_used,
                 waves * WAVE, h->aux_p, tile_queue(h, tiles, waves, st), ck_rows_of(h)};
    if (h->d_simd_prog && hipMemsetAsync(h->d_simd_prog, 0, SIMD_PROG_BYTES, st) == hipSuccess) a.simd_prog = h->d_simd_prog;
    a.tail_flag = h->d_tail;
    a.tail_seq = ++h->tail_seq;
    const int *pm = h->d_perm, *iv = h->d_inv;
    const dim3 grid((waves + DEC_WAVES - 1) / DEC_WAVES);
    hipLaunchKernelGGL((decode_fn)decode_kernel(h->algo, h->N % win_of(h->algo) != 0), grid, dim3(DEC_BLOCK), 0, st,
                       a, pm, iv, (const int *)h->d_used);
    HIPCHK(hipGetLastError());
    return mark_used(h, st);
}

int tdec_tail_gate(tdec_t *h, void *stream) {
    if (!h) return fail(TDEC_EINVAL, "bad tail gate arguments");
    if (!h->tail_seq) return 0;   // no throughput launch yet: nothing to wait for
    Guard g(h->device);
    hipLaunchKernelGGL(k_tail_gate, dim3(1), dim3(WAVE), 0, (hipStream_t)stream, (const unsigned *)h->d_tail,
                       h->tail_seq);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdec_decode_batch_dev(tdec_t *h, int B, const float *d_llr, long llr_stride, int32_t *d_bits, double *d_lfinal,
                          void *stream) {
    if (!h || B < 0) return fail(TDEC_EINVAL, "bad decode arguments");
    if (B == 0) return 0;
    if (B > h->cap_batch) return fail(TDEC_ECAPACITY, "batch larger than tdec_reserve()");
    if (int rc = order_on(h, (hipStream_t)stream)) return rc;   // planes_own may still be read elsewhere
    int rc = tdec_depuncture_dev(h, B, d_llr, llr_stride, (float *)h->planes_own.p, stream);
    if (!rc) rc = tdec_decode_planes_dev(h, B, (const float *)h->planes_own.p, d_bits, d_lfinal, stream);
    return rc;
}

// Zero-copy single calls: a small host-pointer call of at most ZC_MAX_ROWS rows lets the kernels read their
// inputs from, and write their outputs to, the page-locked staging buffer itself
// instead of a DMA each way.  Measured (profiles/r04y/, r04z/): bcjr_max_log_map
// at N = 752 0.065 vs 0.073 ms, one decode() 0.306 vs 0.317 ms, 16 codewords
// 0.352 vs 0.366 ms, 64 even (0.404 vs 0.41), 256 slower (0.677 vs 0.618).
constexpr int ZC_MAX_ROWS = 64;
static bool zero_copy(int B) { return B <= ZC_MAX_ROWS; }


// Host-pointer decode in chunks, so device memory stays bounded for any B:
// by default half the resident-wave capacity (65 536 codewords on MI355X);
// TDEC_HOST_CHUNK overrides it (tests use a small value to exercise the chunk
// loop).  Three streams and two alternating device buffers per direction:
// uploads (h->cstream), decodes (h->stream) and downloads (h->dstream), so the
// upload of chunk i+1, the decode of chunk i and the download of chunk i-1 run
// at once (the two PCIe directions and the GPU).  With pageable host memory HIP
// stages every copy through its own pinned buffer on the CPU, which caps the
// path at the host's staging rate; host buffers from tdec_host_alloc (or
// registered by the caller) go straight to the DMA engines.
constexpr size_t SMALL_CALL_BYTES = 16u << 20;
struct EventPair {
    hipEvent_t e[2] = {nullptr, nullptr};
    int create() {
        for (auto &x : e)
            if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) return fail(TDEC_EHIP, "hipEventCreate");
        return 0;
    }
    ~EventPair() {
        for (auto &x : e)
            if (x) hipEventDestroy(x);
    }
};

int tdec_decode_batch(tdec_t *h, int B, const float *llr, long llr_stride, int32_t *bits, double *lfinal) {
    if (!h || B < 0) return fail(TDEC_EINVAL, "bad decode arguments");
    if (llr_stride < h->llr_len) return fail(TDEC_ESHORT, "llr rows shorter than the de-puncture walk");
    if (B == 0) return 0;
    if (!llr || !bits) return fail(TDEC_EINVAL, "bad decode arguments");
    Guard g(h->device);
    quiesce(h);   // earlier _dev work on other streams may still use the buffers staged below
    long chunk = std::max(1L, (long)h->max_waves / 2) * WAVE;
    if (const char *pc = getenv("TDEC_HOST_CHUNK")) chunk = std::max(1L, atol(pc));
    const int C = (int)std::min<long>(B, chunk);
    const long n_chunks = (B + C - 1) / C;
    // Small calls (one chunk, <= SMALL_CALL_BYTES of traffic; decode() per frame is
    // 12 KB in and 6 KB out): one page-locked staging buffer, one DMA each way on
    // the handle's stream, no events -- the pageable copies' runtime staging and
    // the pipeline's event setup were most of a per-frame call.
    const size_t in_b = (size_t)B * llr_stride * sizeof(float), bits_b = (size_t)B * 2 * h->N * sizeof(int32_t),
                 lf_b = lfinal ? (size_t)B * 2 * h->N * sizeof(double) : 0;
    // page-locked layout: LLR rows, bits, L_final, each at a 256-B boundary (the
    // zero-copy kernels store int2 / double2 there whatever the row stride)
    auto up256 = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_bits = up256(in_b), o_lf = up256(o_bits + bits_b), pin_b = o_lf + lf_b;
    if (n_chunks == 1 && pin_b <= SMALL_CALL_BYTES) {
        int rc = tdec_reserve(h, B);
        if (!rc) rc = h->h_llr.ensure(in_b);
        if (!rc) rc = h->h_bits.ensure(bits_b);
        if (!rc && lfinal) rc = h->h_lf.ensure(lf_b);
        if (!rc) rc = h->pin.ensure(pin_b);
        if (rc) return rc;
        DrainOnExit drain{h->stream, nullptr};
        char *pin = (char *)h->pin.p;
        std::memcpy(pin, llr, in_b);
        if (zero_copy(B) && use_lowlat(h, B) && use_frame_decoder(h) && h->pin.dev) {
            // zero copy: the de-puncture kernel reads the LLR rows from the page-locked
            // buffer and the frame decoder writes bits / L_final into it
            char *dp = (char *)h->pin.dev;
            if ((rc = tdec_decode_batch_dev(h, B, (const float *)dp, llr_stride, (int32_t *)(dp + o_bits),
                                            lfinal ? (double *)(dp + o_lf) : nullptr, h->stream)))
                return rc;
            HIPCHK(hipStreamSynchronize(h->stream));
            drain.disarm();
            mark_idle(h);
            std::memcpy(bits, pin + o_bits, bits_b);
            if (lfinal) std::memcpy(lfinal, pin + o_lf, lf_b);
            return 0;
        }
        HIPCHK(hipMemcpyAsync(h->h_llr.p, pin, in_b, hipMemcpyHostToDevice, h->stream));
        if ((rc = tdec_decode_batch_dev(h, B, (const float *)h->h_llr.p, llr_stride, (int32_t *)h->h_bits.p,
                                        lfinal ? (double *)h->h_lf.p : nullptr, h->stream)))
            return rc;
        HIPCHK(hipMemcpyAsync(pin + o_bits, h->h_bits.p, bits_b, hipMemcpyDeviceToHost, h->stream));
        if (lfinal) HIPCHK(hipMemcpyAsync(pin + o_lf, h->h_lf.p, lf_b, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        drain.disarm();
        mark_idle(h);
        std::memcpy(bits, pin + o_bits, bits_b);
        if (lfinal) std::memcpy(lfinal, pin + o_lf, lf_b);
        return 0;
    }
    const int nbuf = n_chunks > 1 ? 2 : 1;
    int rc = tdec_reserve(h, C);
    const size_t row_b = (size_t)2 * h->N, llr_c = (size_t)C * llr_stride, bits_c = (size_t)C * row_b;
    if (!rc) rc = h->h_llr.ensure(nbuf * llr_c * sizeof(float));
    if (!rc) rc = h->h_bits.ensure(nbuf * bits_c * sizeof(int32_t));
    if (!rc && lfinal) rc = h->h_lf.ensure(nbuf * bits_c * sizeof(double));
    if (rc) return rc;
    if (nbuf == 2 && !h->cstream) HIPCHK(hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking));
    if (nbuf == 2 && !h->dstream) HIPCHK(hipStreamCreateWithFlags(&h->dstream, hipStreamNonBlocking));
    hipStream_t us = nbuf == 2 ? h->cstream : h->stream, ds = nbuf == 2 ? h->dstream : h->stream;
    EventPair up, dec, down;
    // declared after the events, so it is destroyed (drains the streams) before they are
    struct Drain3 {
        hipStream_t a, b, c;
        ~Drain3() {
            for (hipStream_t s : {a, b, c})
                if (s) hipStreamSynchronize(s);
        }
    } drain{h->stream, us != h->stream ? us : nullptr, ds != h->stream ? ds : nullptr};
    if ((rc = up.create()) || (rc = dec.create()) || (rc = down.create())) return rc;
    float *dl = (float *)h->h_llr.p;
    int32_t *db = (int32_t *)h->h_bits.p;
    double *df = lfinal ? (double *)h->h_lf.p : nullptr;
    auto rows = [&](long i) { return (int)std::min<long>(C, B - i * C); };
    // chunk i: upload into LLR buffer i % 2 (last read by decode i-2), decode into bits
    // buffer i % 2 (last read by download i-2).  Issue order upload(i+1), decode(i+1)
    // before download(i): with pageable memory the runtime performs each copy on this
    // host thread, so the upload of the next chunk overlaps the running decode and the
    // next decode is queued before the host blocks in the download.
    auto stage = [&](long i) -> int {
        const int k = (int)(i % nbuf), n = rows(i);
        if (i >= 2) HIPCHK(hipStreamWaitEvent(us, dec.e[k], 0));
        HIPCHK(hipMemcpyAsync(dl + k * llr_c, llr + i * C * llr_stride, (size_t)n * llr_stride * sizeof(float),
                              hipMemcpyHostToDevice, us));
        HIPCHK(hipEventRecord(up.e[k], us));
        HIPCHK(hipStreamWaitEvent(h->stream, up.e[k], 0));
        if (i >= 2) HIPCHK(hipStreamWaitEvent(h->stream, down.e[k], 0));
        if (int r = tdec_decode_batch_dev(h, n, dl + k * llr_c, llr_stride, db + k * bits_c,
                                          df ? df + k * bits_c : nullptr, h->stream))
            return r;
        HIPCHK(hipEventRecord(dec.e[k], h->stream));
        return 0;
    };
    if ((rc = stage(0))) return rc;
    for (long i = 0; i < n_chunks; ++i) {
        const int k = (int)(i % nbuf), n = rows(i);
        if (i + 1 < n_chunks && (rc = stage(i + 1))) return rc;
        HIPCHK(hipStreamWaitEvent(ds, dec.e[k], 0));
        HIPCHK(hipMemcpyAsync(bits + i * C * row_b, db + k * bits_c, (size_t)n * row_b * sizeof(int32_t),
                              hipMemcpyDeviceToHost, ds));
        if (lfinal)
            HIPCHK(hipMemcpyAsync(lfinal + i * C * row_b, df + k * bits_c, (size_t)n * row_b * sizeof(double),
                                  hipMemcpyDeviceToHost, ds));
        HIPCHK(hipEventRecord(down.e[k], ds));
    }
    HIPCHK(hipStreamSynchronize(ds));
    HIPCHK(hipStreamSynchronize(us));
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
}

// Pinned host memory for the host-pointer entry points (the DMA engines read and
// write it directly; pageable memory is staged by the runtime).
int tdec_host_alloc(size_t bytes, void **out) {
    if (!out) return fail(TDEC_EINVAL, "null argument");
    *out = nullptr;
    if (bytes == 0) return 0;
    HIPCHK(hipHostMalloc(out, bytes, hipHostMallocDefault));
    return 0;
}

void tdec_host_free(void *p) {
    if (p) hipHostFree(p);
}

#if TDEC_FR_STATS
// measurement build only: the frame decoder's block / round counters since the last
// call (blocks of 4 steps: phase A, fix-up rounds, pass 2; rounds: fix-up, pass 2)
int tdec_frame_stats(unsigned long long *out) {
    hipDeviceSynchronize();
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fr_stats), 8 * sizeof(unsigned long long)) != hipSuccess)
        return fail(TDEC_EHIP, "g_fr_stats");
    const unsigned long long z[8] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_fr_stats), z, sizeof(z));
    return 0;
}
#endif

#if TDEC_DM_STATS
// measurement build only: symbols per demap path since the last call (see dm_count)
int tdec_demap_stats(unsigned long long *out) {
    hipDeviceSynchronize();
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dm_stats), 8 * sizeof(unsigned long long)) != hipSuccess)
        return fail(TDEC_EHIP, "g_dm_stats");
    const unsigned long long z[8] = {};
    hipMemcpyToSymbol(HIP_SYMBOL(g_dm_stats), z, sizeof(z));
    return 0;
}
#endif

}  // extern "C"

// One SISO launch over n rows already in device-visible memory (device buffers, or
// the page-locked staging's device view for the zero-copy frame kernel).
template <typename T>
static int siso_launch(tdec_t *h, int n, const T *A, const T *B, const T *W, const T *Y, const double *la,
                       const double *lb, double sf, double *ea, double *eb, bool fr, bool spl, hipStream_t s,
                       unsigned *done = nullptr) {
    constexpr bool F64 = sizeof(T) == 8;
    if (fr) {
        FrSisoArgs fa{n, h->N, A, B, W, Y, la, lb, sf, ea, eb, done, h->siso_seq};
        const bool w1 = fr_wpd(h->N, true) == 1;
        hipLaunchKernelGGL((h->algo ? (w1 ? k_siso_frame<T, 1, 1> : k_siso_frame<T, 1, 2>)
                                    : (w1 ? k_siso_frame<T, 0, 1> : k_siso_frame<T, 0, 2>)),
                           dim3((unsigned)n), dim3(FR_BLOCK), fr_lds(h->N, false).total, s, fa);
        HIPCHK(hipGetLastError());
        return 0;
    }
    const int nwv = n_tiles_of(n);
    if (spl) {   // A/B prototype: one state per lane, 4 codewords per wave (tdec_spl.hip)
        const long sw = (n + 3) / 4;                     // waves
        const long stride = ((h->N + SPL_W - 1) / SPL_W + RING) * 64L;
        if (int rc = h->spl_ck.ensure(sizeof(float) * stride * ((sw + 3) / 4 * 4))) return rc;
        SplArgs sa{n, h->N, (const float *)A, (const float *)B, (const float *)W, (const float *)Y, la, lb, sf, ea, eb,
                   (float *)h->spl_ck.p, stride};
        hipLaunchKernelGGL(k_siso_spl, dim3((unsigned)((sw + 3) / 4)), dim3(256), 0, s, sa);
        HIPCHK(hipGetLastError());
        return 0;
    }
    SisoArgs a{};
    a.B = n, a.N = h->N, a.n_waves = nwv, a.LaA = la, a.LaB = lb, a.sf = sf, a.LeA = ea, a.LeB = eb;
    a.ck = h->ck_p, a.ck_stride = ck_stride_of(h);
    if constexpr (F64) a.Lc64A = A, a.Lc64B = B, a.Lc64W = W, a.Lc64Y = Y;
    else a.LcA = A, a.LcB = B, a.LcW = W, a.LcY = Y;
    const dim3 grid((nwv + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    const bool rag = h->N % WIN != 0;   // the row SISO runs siso<> at WIN
    if (h->algo && rag) hipLaunchKernelGGL((k_siso_batch_logmap<true, F64>), grid, dim3(BLOCK), 0, s, a);
    else if (h->algo) hipLaunchKernelGGL((k_siso_batch_logmap<false, F64>), grid, dim3(BLOCK), 0, s, a);
    else if (rag) hipLaunchKernelGGL((k_siso_batch<true, F64>), grid, dim3(BLOCK), 0, s, a);
    else hipLaunchKernelGGL((k_siso_batch<false, F64>), grid, dim3(BLOCK), 0, s, a);
    HIPCHK(hipGetLastError());
    return 0;
}

// Which SISO kernel serves a handle: max-log rows go to the frame SISO (one row per
// workgroup, tdec_frame.hip; no workspace) unless TDEC_SISO_FRAME=0 (A/B) or its LDS
// does not fit; TDEC_SISO_SPL=1 selects the state-per-lane prototype (float32 only).
// log-MAP rows take the frame SISO up to LM_FRAME_MAX rows per call (the row kernel's
// one lane per row is a serial chain of max* per codeword).
static void siso_route(const tdec_t *h, bool f64, int B, bool &fr, bool &spl) {
    const char *se = getenv("TDEC_SISO_SPL");
    spl = !f64 && se && se[0] == '1' && h->algo == TDEC_ALGO_MAXLOG;
    const char *sfe = getenv("TDEC_SISO_FRAME");
    fr = !spl && (h->algo == TDEC_ALGO_MAXLOG || B <= LM_FRAME_MAX) && !(sfe && sfe[0] == '0') && frame_fits(h->N, false);
}

// tdec_siso_batch / tdec_siso_batch_f64: T = the channel LLRs' dtype.
template <typename T>
static int siso_batch_impl(tdec_t *h, int B, const T *LcA, const T *LcB, const T *LcW, const T *LcY, const double *LaA,
                           const double *LaB, double sf, double *LeA, double *LeB) {
    constexpr bool F64 = sizeof(T) == 8;
    if (!h || B < 0) return fail(TDEC_EINVAL, "bad siso arguments");
    if (B == 0) return 0;
    if (!LcA || !LcB || !LcW || !LcY || !LaA || !LaB || !LeA || !LeB) return fail(TDEC_EINVAL, "bad siso arguments");
    Guard g(h->device);
    quiesce(h);
    DrainOnExit drain{h->stream, nullptr};
    // rows in chunks, like tdec_decode_batch: device memory stays bounded for any B
    long chunk = 4L * h->max_waves * WAVE;
    if (const char *pc = getenv("TDEC_HOST_CHUNK")) chunk = std::max(1L, atol(pc));
    const int C = (int)std::min<long>(B, chunk), waves = n_tiles_of(C);
    const size_t N = h->N, cf = (size_t)C * N * sizeof(T), cd = (size_t)C * N * sizeof(double);
    bool fr, spl;
    siso_route(h, F64, B, fr, spl);
    int rc = fr ? frame_lds_attr(h->device) : ensure_ws(h, waves);
    if (!rc) rc = h->h_misc.ensure(4 * cf + 4 * cd);
    if (rc) return rc;
    char *base = (char *)h->h_misc.p;
    T *dA = (T *)base, *dB = (T *)(base + cf), *dW = (T *)(base + 2 * cf), *dY = (T *)(base + 3 * cf);
    double *daA = (double *)(base + 4 * cf), *daB = (double *)(base + 4 * cf + cd);
    double *deA = (double *)(base + 4 * cf + 2 * cd), *deB = (double *)(base + 4 * cf + 3 * cd);
    hipStream_t s = h->stream;
    // small calls: the six inputs packed into one page-locked buffer laid out as the
    // device staging, one DMA each way
    const bool small = B <= C && 4 * cf + 4 * cd <= SMALL_CALL_BYTES;
    if (small) {
        if (int rc = h->pin.ensure(4 * cf + 4 * cd)) return rc;
    }
    for (long r0 = 0; r0 < B; r0 += C) {
        const int n = (int)std::min<long>(C, B - r0);
        const size_t o = (size_t)r0 * N, nf = (size_t)n * N * sizeof(T), nd = (size_t)n * N * sizeof(double);
        if (small) {
            char *pin = (char *)h->pin.p;
            std::memcpy(pin, LcA + o, nf);
            std::memcpy(pin + cf, LcB + o, nf);
            std::memcpy(pin + 2 * cf, LcW + o, nf);
            std::memcpy(pin + 3 * cf, LcY + o, nf);
            std::memcpy(pin + 4 * cf, LaA + o, nd);
            std::memcpy(pin + 4 * cf + cd, LaB + o, nd);
            if (fr && zero_copy(n) && h->pin.dev) {
                // zero copy: the frame SISO reads its rows from, and writes its
                // extrinsics to, the page-locked buffer itself (each value crosses
                // PCIe once either way: the kernel keeps its inputs in registers):
                // no DMA in either direction
                char *dp = (char *)h->pin.dev;
                if (int rc = siso_launch<T>(h, n, (const T *)dp, (const T *)(dp + cf), (const T *)(dp + 2 * cf),
                                            (const T *)(dp + 3 * cf), (const double *)(dp + 4 * cf),
                                            (const double *)(dp + 4 * cf + cd), sf, (double *)(dp + 4 * cf + 2 * cd),
                                            (double *)(dp + 4 * cf + 3 * cd), true, false, s))
                    return rc;
                HIPCHK(hipStreamSynchronize(s));
                std::memcpy(LeA + o, pin + 4 * cf + 2 * cd, nd);
                std::memcpy(LeB + o, pin + 4 * cf + 3 * cd, nd);
                continue;
            }
            HIPCHK(hipMemcpyAsync(base, pin, 4 * cf + 2 * cd, hipMemcpyHostToDevice, s));
        } else {
            HIPCHK(hipMemcpyAsync(dA, LcA + o, nf, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(dB, LcB + o, nf, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(dW, LcW + o, nf, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(dY, LcY + o, nf, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(daA, LaA + o, nd, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(daB, LaB + o, nd, hipMemcpyHostToDevice, s));
        }
        if (int rc = siso_launch<T>(h, n, dA, dB, dW, dY, daA, daB, sf, deA, deB, fr, spl, s)) return rc;
        if (small) {
            char *pin = (char *)h->pin.p + 4 * cf + 2 * cd;
            HIPCHK(hipMemcpyAsync(pin, deA, 2 * cd, hipMemcpyDeviceToHost, s));   // deB follows deA
            HIPCHK(hipStreamSynchronize(s));
            std::memcpy(LeA + o, pin, nd);
            std::memcpy(LeB + o, pin + cd, nd);
        } else {
            HIPCHK(hipMemcpyAsync(LeA + o, deA, nd, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(LeB + o, deB, nd, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    }
    drain.disarm();   // every chunk ended in a synchronisation of the handle's stream
    mark_idle(h);
    return 0;
}

// The caller-filled staging of small SISO calls: 8 slots [rows][N] of 8-byte
// elements (LcA, LcB, LcW, LcY, LaA, LaB, LeA, LeB), each at a 256-B boundary; a
// float32 channel-LLR row uses the first half of its slot.
static size_t siso_slot(const tdec_t *h, int rows) { return ((size_t)rows * h->N * 8 + 255) / 256 * 256; }

// A zero-copy staged call waits for the frame SISO's per-row completion flags
// (coherent, mapped host memory) instead of the stream: the rows' outputs are in
// the page-locked slots once every flag holds the call's sequence number (a row
// sets its flag after a system-scope release of its stores).  The wait is bounded
// in time (SPIN_LIMIT_S); past it the call falls back to a stream wait and counts
// the fallback (tdec_siso_stats), which the GPU tests require to stay at zero.
constexpr double SPIN_LIMIT_S = 0.25;

template <typename T> static int siso_staged_impl(tdec_t *h, int B, double sf) {
    constexpr bool F64 = sizeof(T) == 8;
    if (!h || B < 1 || B > h->siso_rows || !h->pin_siso.p) return fail(TDEC_EINVAL, "bad staged siso call (tdec_siso_staging first)");
    Guard g(h->device);
    quiesce(h);
    DrainOnExit drain{h->stream, nullptr};
    bool fr, spl;
    siso_route(h, F64, B, fr, spl);
    int rc = fr ? frame_lds_attr(h->device) : ensure_ws(h, n_tiles_of(B));
    const size_t sl = siso_slot(h, h->siso_rows);
    const bool zc = fr && zero_copy(B) && h->pin_siso.dev;
    if (!rc && !zc) rc = h->h_misc.ensure(8 * sl);
    if (rc) return rc;
    hipStream_t s = h->stream;
    char *dp;
    if (zc) {
        dp = (char *)h->pin_siso.dev;   // the kernel reads and writes the page-locked slots
    } else {
        dp = (char *)h->h_misc.p;
        HIPCHK(hipMemcpyAsync(dp, h->pin_siso.p, 6 * sl, hipMemcpyHostToDevice, s));
    }
    volatile unsigned *flags = (volatile unsigned *)h->pin_flags.p;
    const bool spin = zc && h->pin_flags.dev;
    if (spin && ++h->siso_seq == 0) h->siso_seq = 1;   // flags start at 0: never a valid sequence number
    if ((rc = siso_launch<T>(h, B, (const T *)dp, (const T *)(dp + sl), (const T *)(dp + 2 * sl), (const T *)(dp + 3 * sl),
                             (const double *)(dp + 4 * sl), (const double *)(dp + 5 * sl), sf, (double *)(dp + 6 * sl),
                             (double *)(dp + 7 * sl), fr, spl, s, spin ? (unsigned *)h->pin_flags.dev : nullptr)))
        return rc;
    if (spin) {
        // The kernel may still be retiring when this returns; later work on the
        // handle's stream is ordered behind it and nothing it touches afterwards is
        // the caller's.  A kernel that never sets the flags (a fault) is caught by
        // the stream wait once the time limit has passed.
        const auto t0 = std::chrono::steady_clock::now();
        unsigned polls = 0;
        for (int r = 0; r < B; ++r)
            while (flags[r] != h->siso_seq) {
                if ((++polls & 1023u) == 0 &&
                    std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > SPIN_LIMIT_S) {
                    ++h->siso_fallbacks;
                    HIPCHK(hipStreamSynchronize(s));
                    if (flags[r] != h->siso_seq) return fail(TDEC_EHIP, "frame SISO finished without flagging its rows");
                    break;
                }
            }
        drain.disarm();
        mark_idle(h);
        return 0;
    }
    if (dp == (char *)h->h_misc.p)
        HIPCHK(hipMemcpyAsync((char *)h->pin_siso.p + 6 * sl, dp + 6 * sl, 2 * sl, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    drain.disarm();
    mark_idle(h);
    return 0;
}

extern "C" {

int tdec_siso_staging(tdec_t *h, int rows, void **buf, size_t *slot_bytes) {
    if (!h || rows < 1 || !buf || !slot_bytes) return fail(TDEC_EINVAL, "bad siso staging arguments");
    Guard g(h->device);
    if (rows > h->siso_rows) {
        quiesce(h);
        HIPCHK(hipStreamSynchronize(h->stream));   // a flag-waited call's kernel may still be retiring
        h->pin_siso.release();   // the caller's views of the old buffer die with this call
        h->pin_flags.release();
        h->siso_rows = 0;
        if (int rc = h->pin_siso.ensure(8 * siso_slot(h, rows))) return rc;
        // the per-row completion flags (coherent: polled while the kernel runs)
        if (int rc = h->pin_flags.ensure(((size_t)rows * 4 + 255) / 256 * 256, hipHostMallocCoherent | hipHostMallocMapped))
            return rc;
        h->siso_rows = rows;
        std::memset(h->pin_flags.p, 0, (size_t)rows * 4);
    }
    *buf = h->pin_siso.p;
    *slot_bytes = siso_slot(h, h->siso_rows);
    return 0;
}

int tdec_siso_staged(tdec_t *h, int B, int lc_f64, double sf) {
    return lc_f64 ? siso_staged_impl<double>(h, B, sf) : siso_staged_impl<float>(h, B, sf);
}

int tdec_siso_stats(const tdec_t *h, long *flag_fallbacks) {
    if (!h || !flag_fallbacks) return fail(TDEC_EINVAL, "bad siso stats arguments");
    *flag_fallbacks = h->siso_fallbacks;
    return 0;
}

int tdec_siso_batch(tdec_t *h, int B, const float *LcA, const float *LcB, const float *LcW, const float *LcY,
                    const double *LaA, const double *LaB, double sf, double *LeA, double *LeB) {
    return siso_batch_impl<float>(h, B, LcA, LcB, LcW, LcY, LaA, LaB, sf, LeA, LeB);
}

int tdec_siso_batch_f64(tdec_t *h, int B, const double *LcA, const double *LcB, const double *LcW,
                        const double *LcY, const double *LaA, const double *LaB, double sf, double *LeA,
                        double *LeB) {
    return siso_batch_impl<double>(h, B, LcA, LcB, LcW, LcY, LaA, LaB, sf, LeA, LeB);
}

int tdec_demap_dev(int device, const void *d_syms, int sym_f64, long n_sym, const void *cons, int cons_f64, int M,
                   int bps, double noise_var, int div_f32, int sign, double *d_llr, void *stream) {
    if (!d_syms || !cons || !d_llr || n_sym < 0) return fail(TDEC_EINVAL, "bad demap arguments");
    if (int rc = check_demap_args(M, bps)) return rc;
    if (n_sym == 0) return 0;
    Guard g(device);
    const bool f64 = sym_f64 || cons_f64;
    hipStream_t st = (hipStream_t)stream;
    // Tables are cached per (thread, device) by content and never overwritten
    // while another stream may still read them: a new table takes a fresh slot;
    // only when all slots are taken is the oldest reused, after a device-wide
    // synchronisation.
    constexpr int SLOTS = 8;
    static thread_local std::vector<ConsCache> tbl[16];
    static thread_local int next_victim[16];
    std::vector<ConsCache> &v = tbl[device & 15];
    if (v.empty()) v.reserve(SLOTS);
    ConsCache *hit = nullptr;
    for (auto &c : v)
        if (c.matches(cons, cons_f64, M, bps, f64)) hit = &c;
    if (!hit) {
        if ((int)v.size() < SLOTS) {
            v.emplace_back();
            hit = &v.back();
        } else {
            HIPCHK(hipDeviceSynchronize());
            hit = &v[next_victim[device & 15]++ % SLOTS];
        }
    }
    ConsCache &cc = *hit;
    if (int rc = cc.upload(cons, cons_f64, M, bps, f64, st)) return rc;
    DevBuf &tb = cc.buf;
    const DemapCfg c = demap_cfg(M, div_f32, sign, noise_var, cc.sep);
    if (f64) {
        if (sym_f64) return launch_demap<double, double>(bps, (const double *)d_syms, n_sym, (const double *)tb.p, c, d_llr, st);
        return launch_demap<double, float>(bps, (const float *)d_syms, n_sym, (const double *)tb.p, c, d_llr, st);
    }
    return launch_demap<float, float>(bps, (const float *)d_syms, n_sym, (const float *)tb.p, c, d_llr, st);
}

int tdec_demap(int device, const void *syms, int sym_f64, long n_sym, const void *cons, int cons_f64, int M, int bps,
               double noise_var, int div_f32, int sign, double *llr) {
    if (!syms || !cons || !llr || n_sym < 0) return fail(TDEC_EINVAL, "bad demap arguments");
    if (int rc = check_demap_args(M, bps)) return rc;
    if (n_sym == 0) return 0;
    Guard g(device);
    const size_t ns = (size_t)n_sym * 2 * (sym_f64 ? 8 : 4), nl = (size_t)n_sym * bps * sizeof(double);
    void *ds = nullptr, *dl = nullptr;
    HIPCHK(hipMalloc(&ds, ns));
    if (hipMalloc(&dl, nl) != hipSuccess) {
        hipFree(ds);
        return fail(TDEC_ENOMEM, "hipMalloc failed");
    }
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    int rc = 0;
    if (hipMemcpyAsync(ds, syms, ns, hipMemcpyHostToDevice, st) != hipSuccess) rc = fail(TDEC_EHIP, "memcpy");
    if (!rc) rc = tdec_demap_dev(device, ds, sym_f64, n_sym, cons, cons_f64, M, bps, noise_var, div_f32, sign,
                                 (double *)dl, st);
    if (!rc && hipMemcpyAsync(llr, dl, nl, hipMemcpyDeviceToHost, st) != hipSuccess) rc = fail(TDEC_EHIP, "memcpy");
    if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = fail(TDEC_EHIP, "demap failed");
    hipStreamDestroy(st);
    hipFree(ds);
    hipFree(dl);
    return rc;
}

int tdec_selftest(int device, int which, long long n, unsigned long long seed, long long *mismatches) {
    if (!mismatches || which < 0 || which > 4 || n < 0) return fail(TDEC_EINVAL, "bad selftest arguments");
    if (which == 0) n = (1LL << 23) + 1;   // every f32 in [1, 2]
    if (which == 3) n = 0x7F800000LL - 0x42400000LL + 1;   // every f32 t in [48, +inf]
    *mismatches = 0;
    if (n == 0) return 0;
    Guard g(device);
    unsigned long long *d = nullptr;
    HIPCHK(hipMalloc(&d, 2 * sizeof(*d)));
    int rc = 0;
    if (hipMemset(d, 0, 2 * sizeof(*d)) != hipSuccess) rc = fail(TDEC_EHIP, "memset");
    if (!rc) {
        hipLaunchKernelGGL(k_selftest, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, 0, which, n, seed, d);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = fail(TDEC_EHIP, "selftest failed");
    }
    unsigned long long h[2] = {0, 0};
    if (!rc && hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) rc = fail(TDEC_EHIP, "memcpy");
    hipFree(d);
    if (!rc && h[1] != (unsigned long long)n) rc = fail(TDEC_EHIP, "selftest evaluated fewer items than asked");
    *mismatches = (long long)h[0];
    return rc;
}

int tdec_selftest_trans(int device, int which, uint32_t lo_bits, long long n, float *out) {
    if (!out || which < 0 || which > 1 || n < 0 || (unsigned long long)lo_bits + (unsigned long long)n > (1ull << 32))
        return fail(TDEC_EINVAL, "bad selftest_trans arguments");
    if (n == 0) return 0;
    Guard g(device);
    float *d = nullptr;
    HIPCHK(hipMalloc(&d, (size_t)n * sizeof(float)));
    int rc = 0;
    hipLaunchKernelGGL(k_trans_table, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, 0, which, lo_bits, n, d);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = fail(TDEC_EHIP, "selftest_trans failed");
    if (!rc && hipMemcpy(out, d, (size_t)n * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(TDEC_EHIP, "memcpy");
    hipFree(d);
    return rc;
}

int tdec_demap_planes_dev(tdec_t *h, int B, const float *d_syms, int S, const void *cons, int cons_f64, int M,
                          int bps, double noise_var, int div_f32, float *d_planes, void *stream) {
    if (!h || B < 0 || !cons) return fail(TDEC_EINVAL, "bad demap arguments");
    if (int rc = check_demap_args(M, bps)) return rc;
    if (B == 0) return 0;
    if (!d_syms || !d_planes || S <= 0) return fail(TDEC_EINVAL, "bad demap arguments");
    Guard g(h->device);
    hipStream_t st = (hipStream_t)stream;
    if (int rc = order_on(h, st)) return rc;   // the table below may still be read on another stream
    if (int rc = h->cons.upload(cons, cons_f64, M, bps, cons_f64 != 0, st)) return rc;
    const DemapCfg c = demap_cfg(M, div_f32, -1, noise_var, h->cons.sep);
    const long n_avail = std::min<long>((long)S * bps, h->llr_len);   // LLRs the symbols provide
    const int chunks = (h->N + dm_kc(bps) - 1) / dm_kc(bps);
    const long n_items = (long)n_tiles_of(B) * chunks;   // (64-codeword tile, dm_kc-couple chunk) pairs
    float *P = d_planes;
    const long n_tiles = n_tiles_of(B);
    DemapDecl dd{h->d_decl, h->d_decl_n, h->d_decl_ovf, DM_DECL_CAP};
    const bool split = dm_split_table(bps, h->cons.sep);
    if (split) {   // the decline list: sized by tdec_reserve / tdec_reserve_fused
        if (h->decl_tiles < n_tiles) {
            // an unreserved batch: allocate here, outside any stream capture (hipFree
            // synchronises the device, and a captured graph must not hold a buffer
            // freed by a later regrowth)
            if (capturing(st)) return fail(TDEC_ECAPACITY, "demap batch larger than tdec_reserve() (stream capture)");
            quiesce(h);
            if (int rc = ensure_decl(h, n_tiles)) return rc;
        }
        dd = DemapDecl{h->d_decl, h->d_decl_n, h->d_decl_ovf, DM_DECL_CAP};
        HIPCHK(hipMemsetAsync(h->d_decl_n, 0, sizeof(unsigned), st));
        HIPCHK(hipMemsetAsync(h->d_decl_ovf, 0, (size_t)n_tiles, st));
    }
    const dim3 grid((unsigned)n_items);   // one block per item
    const dim3 fgrid((unsigned)std::max<long>(1, std::min<long>(n_tiles, 1024)));
    switch (bps) {
#define LAUNCH_PLANES(TT, K, SP, F64)                                                                     \
    hipLaunchKernelGGL((k_demap_planes<TT, K, SP>), grid, dim3(BLOCK),                                  \
                       0, st, B, h->N, S, d_syms, (const TT *)h->cons.buf.p, c, (const int *)h->d_src,          \
                       (const int *)h->d_off, n_avail, P, n_items, dd)
#define CASE(K)                                                                                              \
    case K:                                                                                                  \
        if (cons_f64) {                                                                                      \
            if constexpr (dm_split(K)) {                                                                     \
                if (split) {                                                                                 \
                    LAUNCH_PLANES(double, K, dm_split(K), 1);                                                \
                    hipLaunchKernelGGL((k_demap_fix<double, K>), fgrid, dim3(BLOCK), 0, st, B, h->N, S, d_syms, \
                                       (const double *)h->cons.buf.p, c, (const int *)h->d_dst, n_avail, P, dd, \
                                       n_tiles);                                                             \
                    break;                                                                                   \
                }                                                                                            \
            }                                                                                                \
            LAUNCH_PLANES(double, K, false, 1);                                                              \
        } else {                                                                                             \
            if constexpr (dm_split(K)) {                                                                     \
                if (split) {                                                                                 \
                    LAUNCH_PLANES(float, K, dm_split(K), 0);                                                 \
                    hipLaunchKernelGGL((k_demap_fix<float, K>), fgrid, dim3(BLOCK), 0, st, B, h->N, S, d_syms,  \
                                       (const float *)h->cons.buf.p, c, (const int *)h->d_dst, n_avail, P, dd,  \
                                       n_tiles);                                                             \
                    break;                                                                                   \
                }                                                                                            \
            }                                                                                                \
            LAUNCH_PLANES(float, K, false, 0);                                                               \
        }                                                                                                    \
        break;
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
#undef CASE
#undef LAUNCH_PLANES
    default: return fail(TDEC_EINVAL, "bps must be 1..8");
    }
    HIPCHK(hipGetLastError());
    return mark_used(h, st);
}

}  // extern "C"

// Workload arguments common to the staged encoder kernel's uses.
static WorkloadArgs workload_args(const tdec_t *h, int B) {
    WorkloadArgs a{};
    a.B = B;
    a.N = h->N;
    a.period = h->period;
    a.n_out = h->enc_len;
    std::memcpy(a.punct, h->punct, 16);
    std::memcpy(a.circ, h->circ, sizeof a.circ);
    a.perm = h->d_perm;
    return a;
}
static bool staged_encoder_ok(const tdec_t *h) { return h->N % 4 == 0 && h->N <= ENC_MAX_N; }

extern "C" {

int tdec_workload_dev(tdec_t *h, int B, int64_t cw0, uint64_t seed, const float *cons_iq, int M, int bps,
                      double sigma, float *d_syms, uint8_t *d_info, void *stream) {
    if (!h || B < 0 || cw0 < 0) return fail(TDEC_EINVAL, "bad workload arguments");
    if (B == 0) return 0;
    // every bps-bit label indexes the table, so it must hold all 2^bps points
    if (!cons_iq || !d_syms || bps < 1 || bps > 8 || M != (1 << bps) || !(sigma >= 0.0))
        return fail(TDEC_EINVAL, "bad workload arguments (the constellation must have 2^bps points)");
    if (!staged_encoder_ok(h)) return fail(TDEC_EINVAL, "workload generation needs N % 4 == 0 and N <= 1024");
    Guard g(h->device);
    WorkloadArgs a = workload_args(h, B);
    a.bps = bps;
    a.M = M;
    a.S = (int)((h->enc_len + bps - 1) / bps);
    a.cw0 = (uint64_t)cw0;
    a.seed = seed;
    a.sigma = (float)sigma;
    for (int m = 0; m < M; ++m) a.cons[m] = make_float2(cons_iq[2 * m], cons_iq[2 * m + 1]);
    a.info_out = d_info;
    a.syms = reinterpret_cast<float2 *>(d_syms);
    hipLaunchKernelGGL(k_workload, dim3((unsigned)n_tiles_of(B)), dim3(64), 0, (hipStream_t)stream, a);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdec_info_bits_dev(tdec_t *h, int B, int64_t cw0, uint64_t seed, uint8_t *d_info, void *stream) {
    if (!h || B < 0 || cw0 < 0) return fail(TDEC_EINVAL, "bad info-bits arguments");
    if (B == 0) return 0;
    if (!d_info) return fail(TDEC_EINVAL, "bad info-bits arguments");
    if (!staged_encoder_ok(h)) return fail(TDEC_EINVAL, "workload generation needs N % 4 == 0 and N <= 1024");
    Guard g(h->device);
    WorkloadArgs a = workload_args(h, B);
    a.cw0 = (uint64_t)cw0;
    a.seed = seed;
    a.info_out = d_info;
    hipLaunchKernelGGL(k_workload, dim3((unsigned)n_tiles_of(B)), dim3(64), 0, (hipStream_t)stream, a);
    HIPCHK(hipGetLastError());
    return 0;
}

int tdec_count_errors_dev(tdec_t *h, int B, int64_t cw0, uint64_t seed, const int32_t *d_bits, int32_t *d_errs,
                          void *stream) {
    if (!h || B < 0 || cw0 < 0) return fail(TDEC_EINVAL, "bad count-errors arguments");
    if (B == 0) return 0;
    if (!d_bits || !d_errs) return fail(TDEC_EINVAL, "bad count-errors arguments");
    Guard g(h->device);
    hipLaunchKernelGGL(k_count_errors, dim3((unsigned)B), dim3(64), 0, (hipStream_t)stream, B, h->N, (uint64_t)cw0,
                       seed, d_bits, d_errs);
    HIPCHK(hipGetLastError());
    return 0;
}

// ---- fused demap + decode (k_turbo_decode_syms) ---------------------------------------
typedef void (*fused_fn)(DecodeArgs, const int *, const int *, const int *, FusedDemapArgs);

// The instantiated (algorithm, symbol dtype, bits per symbol) combinations: the
// BASELINE configurations (QPSK / 16QAM / 256QAM max-log, 8PSK log-MAP); anything
// else runs k_demap_planes + k_turbo_decode.
static const void *fused_kernel(int algo, bool ragged, bool f64, int bps) {
    if (ragged) return nullptr;
    if (algo == 0 && !f64 && bps == 4) return (const void *)k_turbo_decode_syms<0, false, float, 4>;
    if (algo == 0 && !f64 && bps == 8) return (const void *)k_turbo_decode_syms<0, false, float, 8>;
    if (algo == 0 && f64 && bps == 2) return (const void *)k_turbo_decode_syms<0, false, double, 2>;
    if (algo == 1 && !f64 && bps == 3) return (const void *)k_turbo_decode_syms<1, false, float, 3>;
    return nullptr;
}

static int waves_for(const tdec_t *h, int B) { return std::min(n_tiles_of(B), h->max_waves); }

int tdec_reserve_fused(tdec_t *h, int max_batch) {
    if (!h || max_batch < 0) return fail(TDEC_EINVAL, "bad reserve");
    if (max_batch == 0) return 0;
    Guard g(h->device);
    const int w = waves_for(h, max_batch);
    const size_t pw = 2 * (size_t)w * tile_floats(h->N) * sizeof(float);
    if (w > h->ws_waves || pw > h->planes_w.cap) quiesce(h);
    int rc = ensure_ws(h, w);
    if (!rc) rc = h->planes_w.ensure(pw);
    return rc;
}

int tdec_fused_available(const tdec_t *h, int cons_f64, int bps) {
    return h && fused_kernel(h->algo, h->N % win_unstaged(h->algo) != 0, cons_f64 != 0, bps) != nullptr;
}

int tdec_demap_decode_dev(tdec_t *h, int B, const float *d_syms, int S, const void *cons, int cons_f64, int M,
                          int bps, double noise_var, int div_f32, int32_t *d_bits, double *d_lfinal, void *stream) {
    if (!h || B < 0 || !cons) return fail(TDEC_EINVAL, "bad demap-decode arguments");
    if (int rc = check_demap_args(M, bps)) return rc;
    if (B == 0) return 0;
    if (!d_syms || !d_bits || S <= 0) return fail(TDEC_EINVAL, "bad demap-decode arguments");
    const void *k = fused_kernel(h->algo, h->N % win_unstaged(h->algo) != 0, cons_f64 != 0, bps);
    if (!k) return fail(TDEC_EUNSUPPORTED, "no fused demap-decode kernel for this modulation / algorithm");
    Guard g(h->device);
    const int tiles = n_tiles_of(B), waves = waves_for(h, B);
    if (waves > h->ws_waves || 2 * (size_t)waves * tile_floats(h->N) * sizeof(float) > h->planes_w.cap)
        return fail(TDEC_ECAPACITY, "workspace too small: call tdec_reserve_fused first");
    hipStream_t st = (hipStream_t)stream;
    if (int rc = order_on(h, st)) return rc;
    if (int rc = h->cons.upload(cons, cons_f64, M, bps, cons_f64 != 0, st)) return rc;
    DecodeArgs a{B, h->N, h->iters, tiles, waves, nullptr, h->le_p, h->ck_p, d_bits, d_lfinal, h->d_used,
                 waves * WAVE, h->aux_p, tile_queue(h, tiles, waves, st), ck_rows_of(h)};
    FusedDemapArgs fa{d_syms, S, std::min<long>((long)S * bps, h->llr_len), (const int *)h->d_src,
                      (const int *)h->d_off, (float *)h->planes_w.p,
                      demap_cfg(M, div_f32, -1, noise_var, h->cons.sep), h->cons.buf.p};
    const dim3 grid((waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK);
    hipLaunchKernelGGL((fused_fn)k, grid, dim3(BLOCK), 0, st, a, (const int *)h->d_perm, (const int *)h->d_inv,
                       (const int *)h->d_used, fa);
    HIPCHK(hipGetLastError());
    return mark_used(h, st);
}

int tdec_encode_dev(tdec_t *h, int B, const uint8_t *d_bits, uint8_t *d_coded, void *stream) {
    if (!h || B < 0) return fail(TDEC_EINVAL, "bad encode arguments");
    if (B == 0) return 0;
    if (!d_bits || !d_coded) return fail(TDEC_EINVAL, "bad encode arguments");
    Guard g(h->device);
    if (staged_encoder_ok(h)) {   // coalesced LDS-staged encoder (tdec_workload.hip)
        WorkloadArgs w = workload_args(h, B);
        w.bits_in = d_bits;
        w.coded_out = d_coded;
        hipLaunchKernelGGL(k_workload, dim3((unsigned)n_tiles_of(B)), dim3(64), 0, (hipStream_t)stream, w);
        HIPCHK(hipGetLastError());
        return 0;
    }
    EncodeArgs a{};
    a.B = B;
    a.N = h->N;
    a.period = h->period;
    a.n_out = h->enc_len;
    std::memcpy(a.punct, h->punct, 16);
    std::memcpy(a.circ, h->circ, sizeof a.circ);
    a.perm = h->d_perm;
    a.bits = d_bits;
    a.coded = d_coded;
    hipLaunchKernelGGL(k_encode, dim3((B + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, (hipStream_t)stream, a);
    HIPCHK(hipGetLastError());
    return 0;
}

}  // extern "C"

// ---- built-in Gray constellations and the fixed-signature demapper --------------------
// The label-ordered tables compute_llr builds (test_sdr_with_coding.py:207-208)
// from the reference mappers, with numpy's arithmetic and result dtype:
//   BPSK   2.0 * complex64(b) - 1.0                       (:25-26)          complex64
//   QPSK   complex64(1-2b0 + j(1-2b1)) / np.sqrt(2)        (:31-37)          complex128
//          (numpy divides by the complex128 scalar sqrt(2)+0j with Smith's
//          method: re * (1 / sqrt(2)))
//   8PSK   exp(j * GRAY3[label] * pi / 4) -> complex64    (:45-57)
//   QAM    (2*gray[i] - (L-1)) / sqrt(scale) per axis     (:72-86, sdr_modem.py:142-207) complex64
static int builtin_constellation(int mod, double *iq, int *is_f64) {
    static const int g2[4] = {0, 1, 3, 2}, g3[8] = {0, 1, 3, 2, 6, 7, 5, 4},
                     g4[16] = {0, 1, 3, 2, 6, 7, 5, 4, 12, 13, 15, 14, 10, 11, 9, 8};
    *is_f64 = 0;
    switch (mod) {
    case TDEC_MOD_BPSK:
        for (int i = 0; i < 2; ++i) {
            iq[2 * i] = (double)(2.0f * (float)i - 1.0f);
            iq[2 * i + 1] = 0.0;
        }
        return 2;
    case TDEC_MOD_QPSK: {
        *is_f64 = 1;
        const double scl = 1.0 / (std::sqrt(2.0) + 0.0 * 0.0);
        for (int i = 0; i < 4; ++i) {
            const double re = 1 - 2 * (i >> 1), im = 1 - 2 * (i & 1);
            iq[2 * i] = (re + im * 0.0) * scl;
            iq[2 * i + 1] = (im - re * 0.0) * scl;
        }
        return 4;
    }
    case TDEC_MOD_8PSK:
        for (int i = 0; i < 8; ++i) {
            const double p = g3[i] * M_PI / 4;
            iq[2 * i] = (double)(float)std::cos(p);
            iq[2 * i + 1] = (double)(float)std::sin(p);
        }
        return 8;
    case TDEC_MOD_16QAM:
    case TDEC_MOD_64QAM:
    case TDEC_MOD_256QAM: {
        const int k = mod == TDEC_MOD_16QAM ? 2 : (mod == TDEC_MOD_64QAM ? 3 : 4);
        const int L = 1 << k, scale = k == 2 ? 10 : (k == 3 ? 42 : 170);
        const int *g = k == 2 ? g2 : (k == 3 ? g3 : g4);
        const double sq = std::sqrt((double)scale);
        for (int i = 0; i < L * L; ++i) {
            iq[2 * i] = (double)(float)((double)(2 * g[i >> k] - (L - 1)) / sq);
            iq[2 * i + 1] = (double)(float)((double)(2 * g[i & (L - 1)] - (L - 1)) / sq);
        }
        return L * L;
    }
    default: return fail(TDEC_EINVAL, "unknown modulation id");
    }
}

int tdec_constellation(int mod, double *iq, int *is_f64) {
    if (!iq || !is_f64) return fail(TDEC_EINVAL, "null argument");
    return builtin_constellation(mod, iq, is_f64);
}

int tdec_demap_batch(int device, int mod, int sign, const float *syms_iq, long n_sym, float noise_var,
                     float *llr_out) {
    double tab[512];
    int f64 = 0;
    const int M = builtin_constellation(mod, tab, &f64);
    if (M < 0) return M;
    if (n_sym < 0 || (sign != 1 && sign != -1)) return fail(TDEC_EINVAL, "bad demap arguments");
    int bps = 0;
    while ((1 << bps) < M) ++bps;
    if (n_sym == 0) return 0;
    if (!syms_iq || !llr_out) return fail(TDEC_EINVAL, "bad demap arguments");
    std::vector<float> t32;
    const void *cons = tab;
    if (!f64) {   // complex64 table
        t32.assign(tab, tab + 2 * M);
        cons = t32.data();
    }
    // compute_llr with a Python-float noise_var: the final division stays
    // float32 unless the arithmetic is complex128 (QPSK)
    const double nv = (double)noise_var;
    std::vector<double> l64((size_t)n_sym * bps);
    const int rc = tdec_demap(device, syms_iq, 0, n_sym, cons, f64, M, bps, nv, !f64, sign, l64.data());
    if (rc) return rc;
    for (size_t i = 0; i < l64.size(); ++i) llr_out[i] = (float)l64[i];   // decode()'s f32 cast (:466)
    return 0;
}
