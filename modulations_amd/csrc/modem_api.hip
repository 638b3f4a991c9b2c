// modem_api.hip -- the C ABI (include/modem.h) over modem_kernels.hip.
//
// _dev entry points are stream-ordered and allocation free; tables and taps
// travel by value in the kernel arguments (no upload, no synchronisation).
// Host entry points stage through temporary device buffers on a private
// stream and synchronise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "modem.h"
#include "modem_kernels.hip"

using namespace mdm;

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
            return fail(e_ == hipErrorOutOfMemory ? MDM_ENOMEM : MDM_EHIP,                    \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

struct Guard {
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

// Grid for a grid-stride elementwise pass: enough blocks to fill 256 CUs
// several times over, never more than the work.
dim3 grid_for(long n) {
    long b = (n + BLOCK - 1) / BLOCK;
    if (b > 256L * 16) b = 256L * 16;
    return dim3((unsigned)(b < 1 ? 1 : b));
}

int launch_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MDM_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return 0;
}

// Host staging: device buffers + private stream, freed on scope exit.
struct Stage {
    void *p[3] = {nullptr, nullptr, nullptr};
    hipStream_t st = nullptr;
    int init() {
        HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        return 0;
    }
    int alloc(int i, size_t bytes) {
        HIPCHK(hipMalloc(&p[i], bytes ? bytes : 1));
        return 0;
    }
    int h2d(int i, const void *src, size_t bytes) {
        if (bytes) HIPCHK(hipMemcpyAsync(p[i], src, bytes, hipMemcpyHostToDevice, st));
        return 0;
    }
    int d2h(void *dst, int i, size_t bytes) {
        if (bytes) HIPCHK(hipMemcpyAsync(dst, p[i], bytes, hipMemcpyDeviceToHost, st));
        return 0;
    }
    int sync() {
        HIPCHK(hipStreamSynchronize(st));
        return 0;
    }
    ~Stage() {
        for (void *q : p)
            if (q) hipFree(q);
        if (st) hipStreamDestroy(st);
    }
};

}  // namespace

extern "C" {

const char *mdm_last_error(void) { return g_err.c_str(); }

// ---------------------------------------------------------------- mapper -----------------
int mdm_map_dev(int device, const uint8_t *d_bits, long n_bits, int bps, const void *table, int table_f64,
                void *d_syms, void *stream) {
    if (n_bits < 0 || bps < 1 || bps > 8 || !table) return fail(MDM_EINVAL, "bad mapper arguments");
    if (table_f64 && bps > 7) return fail(MDM_EINVAL, "complex128 mapper tables hold at most 128 points");
    if (n_bits == 0) return 0;
    if (!d_bits || !d_syms) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    MapTable t;
    std::memset(&t, 0, sizeof t);
    std::memcpy(table_f64 ? (void *)t.d : (void *)t.f, table, (size_t)(2 << bps) * (table_f64 ? 8 : 4));
    const long n_sym = (n_bits + bps - 1) / bps;
    hipStream_t st = (hipStream_t)stream;
    long nblk = (n_sym + MAP_SPB - 1) / MAP_SPB;
    const dim3 grid((unsigned)(nblk < 256L * 8 ? nblk : 256L * 8));
    if (table_f64)
        hipLaunchKernelGGL((k_map<double>), grid, dim3(BLOCK), 0, st, d_bits, n_bits, bps, n_sym, t, (double2 *)d_syms);
    else
        hipLaunchKernelGGL((k_map<float>), grid, dim3(BLOCK), 0, st, d_bits, n_bits, bps, n_sym, t, (float2 *)d_syms);
    return launch_check("k_map");
}

int mdm_map(int device, const uint8_t *bits, long n_bits, int bps, const void *table, int table_f64, void *syms) {
    if (n_bits < 0 || bps < 1 || bps > 8 || !table) return fail(MDM_EINVAL, "bad mapper arguments");
    if (n_bits == 0) return 0;
    if (!bits || !syms) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    const long n_sym = (n_bits + bps - 1) / bps;
    const size_t ob = (size_t)n_sym * (table_f64 ? 16 : 8);
    Stage s;
    int rc;
    if ((rc = s.init()) || (rc = s.alloc(0, (size_t)n_bits)) || (rc = s.alloc(1, ob)) ||
        (rc = s.h2d(0, bits, (size_t)n_bits)))
        return rc;
    if ((rc = mdm_map_dev(device, (const uint8_t *)s.p[0], n_bits, bps, table, table_f64, s.p[1], s.st))) return rc;
    if ((rc = s.d2h(syms, 1, ob))) return rc;
    return s.sync();
}

// ---------------------------------------------------------------- hard demod ---------------
static int demod_args(int kind, int bps, const int32_t *labels, double scale, const double *cons, int nan_raises,
                      DemodArgs &a) {
    std::memset(&a, 0, sizeof a);
    a.kind = kind;
    a.bps = bps;
    a.nan_raises = nan_raises ? 1 : 0;
    a.scale = scale;
    int want = 0;
    switch (kind) {
    case MDM_DEMOD_GT0: if (bps != 1) return fail(MDM_EINVAL, "GT0 demod has bps 1"); break;
    case MDM_DEMOD_QPSK: if (bps != 2) return fail(MDM_EINVAL, "QPSK demod has bps 2"); break;
    case MDM_DEMOD_PSK8:
        if (bps != 3) return fail(MDM_EINVAL, "8PSK demod has bps 3");
        want = 8;
        break;
    case MDM_DEMOD_QAM_AXIS:
        if (bps < 2 || bps > 16 || bps % 2) return fail(MDM_EINVAL, "QAM demod needs an even bps");
        a.levels = 1 << (bps / 2);
        if (a.levels > 256) return fail(MDM_EINVAL, "too many QAM levels");
        want = a.levels;
        break;
    case MDM_DEMOD_ARGMIN:
        if (bps < 1 || (1 << bps) > ARG_MAX) return fail(MDM_EINVAL, "argmin demod supports up to 64 points");
        if (!cons) return fail(MDM_EINVAL, "argmin demod needs a constellation");
        std::memcpy(a.cons, cons, sizeof(double) * 2 * (1 << bps));
        break;
    default: return fail(MDM_EINVAL, "unknown demodulator kind");
    }
    for (int i = 0; i < want; ++i) {
        a.labels[i] = labels ? labels[i] : i;
        if (a.labels[i] < 0 || a.labels[i] >= want) return fail(MDM_EINVAL, "label table out of range");
    }
    return 0;
}

int mdm_demod_dev(int device, int kind, const void *d_syms, int sym_f64, long n_sym, int bps, const int32_t *labels,
                  double scale, const double *cons, int nan_raises, uint8_t *d_bits, uint32_t *d_nan_count,
                  void *stream) {
    if (n_sym < 0) return fail(MDM_EINVAL, "negative symbol count");
    DemodArgs a;
    if (int rc = demod_args(kind, bps, labels, scale, cons, nan_raises, a)) return rc;
    if (n_sym == 0) return 0;
    if (!d_syms || !d_bits) return fail(MDM_EINVAL, "null buffer");
    a.vec = ((uintptr_t)d_bits % bps) == 0;
    Guard g(device);
    hipStream_t st = (hipStream_t)stream;
    if (sym_f64)
        hipLaunchKernelGGL((k_demod<double>), grid_for(n_sym), dim3(BLOCK), 0, st, (const double2 *)d_syms, n_sym, a,
                           d_bits, d_nan_count);
    else
        hipLaunchKernelGGL((k_demod<float>), grid_for(n_sym), dim3(BLOCK), 0, st, (const float2 *)d_syms, n_sym, a,
                           d_bits, d_nan_count);
    return launch_check("k_demod");
}

int mdm_demod(int device, int kind, const void *syms, int sym_f64, long n_sym, int bps, const int32_t *labels,
              double scale, const double *cons, int nan_raises, uint8_t *bits) {
    if (n_sym < 0) return fail(MDM_EINVAL, "negative symbol count");
    DemodArgs a;
    if (int rc = demod_args(kind, bps, labels, scale, cons, nan_raises, a)) return rc;
    if (n_sym == 0) return 0;
    if (!syms || !bits) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    const size_t ib = (size_t)n_sym * (sym_f64 ? 16 : 8), ob = (size_t)n_sym * bps;
    Stage s;
    int rc;
    if ((rc = s.init()) || (rc = s.alloc(0, ib)) || (rc = s.alloc(1, ob)) || (rc = s.alloc(2, 4)) ||
        (rc = s.h2d(0, syms, ib)))
        return rc;
    HIPCHK(hipMemsetAsync(s.p[2], 0, 4, s.st));
    if ((rc = mdm_demod_dev(device, kind, s.p[0], sym_f64, n_sym, bps, labels, scale, cons, nan_raises,
                            (uint8_t *)s.p[1], (uint32_t *)s.p[2], s.st)))
        return rc;
    uint32_t nans = 0;
    if ((rc = s.d2h(bits, 1, ob)) || (rc = s.d2h(&nans, 2, 4)) || (rc = s.sync())) return rc;
    if (nans) return fail(MDM_ENAN, "cannot convert float NaN to integer");
    return 0;
}

// ---------------------------------------------------------------- FIR ----------------------
static int fir_plan(long n_x, int n_taps, int up, int down, long offset, long n_out, FirArgs &a, bool &stage,
                    long &blocks) {
    if (n_x < 1 || n_taps < 1 || n_taps > TAPS_MAX || up < 1 || down < 1 || offset < 0 || n_out < 0)
        return fail(MDM_EINVAL, "bad FIR arguments");
    a.n_taps = n_taps;
    a.up = up;
    a.down = down;
    a.off = offset;
    a.n_out = n_out;
    a.n_x = n_x;
    if ((n_out - 1) * down + offset + n_taps >= (1L << 31) || n_x * (long)up + n_taps >= (1L << 31))
        return fail(MDM_EINVAL, "FIR too long for one call (2^31 samples)");
    a.per_thread = down == 1 ? 4 : 1;
    const long opb = (long)BLOCK * a.per_thread;
    const long span = ((opb - 1) * down + n_taps - 1) / up + 2;   // staged samples per block (upper bound)
    stage = span <= FIR_LDS;
    blocks = (n_out + opb - 1) / opb;
    return 0;
}

int mdm_fir_dev(int device, const void *d_x, int x_f64, long n_x, const double *taps, int n_taps, int up, int down,
                long offset, long n_out, double *d_out, void *stream) {
    FirArgs a;
    bool stage;
    long blocks;
    if (!taps) return fail(MDM_EINVAL, "null taps");
    if (int rc = fir_plan(n_x, n_taps, up, down, offset, n_out, a, stage, blocks)) return rc;
    if (n_out == 0) return 0;
    if (!d_x || !d_out) return fail(MDM_EINVAL, "null buffer");
    if (blocks > 0x7fffffffL) return fail(MDM_EINVAL, "FIR output too long");
    std::memset(a.h, 0, sizeof a.h);
    std::memcpy(a.h, taps, sizeof(double) * n_taps);
    Guard g(device);
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)blocks);
    double2 *o = (double2 *)d_out;
    // polyphase up-sampler / phase-major decimator for the shapes the reference uses
    if (down == 1 && (up == 2 || up == 4 || up == 8 || up == 16)) {
        const long nper = (n_out - 1 + offset) / up + 1;
        const dim3 g2((unsigned)std::min<long>((nper + BLOCK - 1) / BLOCK, 256L * 16));
#define UPC(U)                                                                                                  \
    case U:                                                                                                     \
        if (x_f64) hipLaunchKernelGGL((k_fir_up<double, U>), g2, dim3(BLOCK), 0, st, (const double2 *)d_x, a, o); \
        else hipLaunchKernelGGL((k_fir_up<float, U>), g2, dim3(BLOCK), 0, st, (const float2 *)d_x, a, o);         \
        break;
        switch (up) { UPC(2) UPC(4) UPC(8) UPC(16) }
#undef UPC
        return launch_check("k_fir_up");
    }
    if (up == 1 && (down == 1 || down == 2 || down == 4 || down == 8)) {
        const dim3 g2((unsigned)std::min<long>((n_out + BLOCK - 1) / BLOCK, 256L * 16));
#define DNC(D)                                                                                                    \
    case D:                                                                                                       \
        if (x_f64) hipLaunchKernelGGL((k_fir_dec<double, D>), g2, dim3(BLOCK), 0, st, (const double2 *)d_x, a, o); \
        else hipLaunchKernelGGL((k_fir_dec<float, D>), g2, dim3(BLOCK), 0, st, (const float2 *)d_x, a, o);         \
        break;
        switch (down) { DNC(1) DNC(2) DNC(4) DNC(8) }
#undef DNC
        return launch_check("k_fir_dec");
    }
    if (x_f64 && stage) hipLaunchKernelGGL((k_fir<double, true>), grid, dim3(BLOCK), 0, st, (const double2 *)d_x, a, o);
    else if (x_f64) hipLaunchKernelGGL((k_fir<double, false>), grid, dim3(BLOCK), 0, st, (const double2 *)d_x, a, o);
    else if (stage) hipLaunchKernelGGL((k_fir<float, true>), grid, dim3(BLOCK), 0, st, (const float2 *)d_x, a, o);
    else hipLaunchKernelGGL((k_fir<float, false>), grid, dim3(BLOCK), 0, st, (const float2 *)d_x, a, o);
    return launch_check("k_fir");
}

int mdm_fir(int device, const void *x, int x_f64, long n_x, const double *taps, int n_taps, int up, int down,
            long offset, long n_out, double *out) {
    FirArgs a;
    bool stage;
    long blocks;
    if (!taps) return fail(MDM_EINVAL, "null taps");
    if (int rc = fir_plan(n_x, n_taps, up, down, offset, n_out, a, stage, blocks)) return rc;
    if (n_out == 0) return 0;
    if (!x || !out) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    const size_t ib = (size_t)n_x * (x_f64 ? 16 : 8), ob = (size_t)n_out * 16;
    Stage s;
    int rc;
    if ((rc = s.init()) || (rc = s.alloc(0, ib)) || (rc = s.alloc(1, ob)) || (rc = s.h2d(0, x, ib))) return rc;
    if ((rc = mdm_fir_dev(device, s.p[0], x_f64, n_x, taps, n_taps, up, down, offset, n_out, (double *)s.p[1], s.st)))
        return rc;
    if ((rc = s.d2h(out, 1, ob))) return rc;
    return s.sync();
}

// ---------------------------------------------------------------- IQ samples ---------------
int mdm_iq_quantize_dev(int device, const void *d_sig, int sig_f64, long n, int8_t *d_iq, void *d_scratch,
                        void *stream) {
    if (n < 1) return fail(MDM_EINVAL, "zero-size array to reduction operation maximum which has no identity");
    if (!d_sig || !d_iq || !d_scratch) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    hipStream_t st = (hipStream_t)stream;
    unsigned long long *mx = (unsigned long long *)d_scratch;
    HIPCHK(hipMemsetAsync(mx, 0, 8, st));
    if (sig_f64) {
        hipLaunchKernelGGL((k_absmax<double>), grid_for(n), dim3(BLOCK), 0, st, (const double2 *)d_sig, n, mx);
        hipLaunchKernelGGL((k_quantize<double>), grid_for(n), dim3(BLOCK), 0, st, (const double2 *)d_sig, n, mx,
                           (char2 *)d_iq);
    } else {
        hipLaunchKernelGGL((k_absmax<float>), grid_for(n), dim3(BLOCK), 0, st, (const float2 *)d_sig, n, mx);
        hipLaunchKernelGGL((k_quantize<float>), grid_for(n), dim3(BLOCK), 0, st, (const float2 *)d_sig, n, mx,
                           (char2 *)d_iq);
    }
    return launch_check("k_quantize");
}

int mdm_iq_quantize(int device, const void *sig, int sig_f64, long n, int8_t *iq) {
    if (n < 1) return fail(MDM_EINVAL, "zero-size array to reduction operation maximum which has no identity");
    if (!sig || !iq) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    const size_t ib = (size_t)n * (sig_f64 ? 16 : 8), ob = (size_t)n * 2;
    Stage s;
    int rc;
    if ((rc = s.init()) || (rc = s.alloc(0, ib)) || (rc = s.alloc(1, ob)) || (rc = s.alloc(2, 8)) ||
        (rc = s.h2d(0, sig, ib)))
        return rc;
    if ((rc = mdm_iq_quantize_dev(device, s.p[0], sig_f64, n, (int8_t *)s.p[1], s.p[2], s.st))) return rc;
    if ((rc = s.d2h(iq, 1, ob))) return rc;
    return s.sync();
}

int mdm_iq_dequantize_dev(int device, const uint8_t *d_raw, long n_pairs, float *d_sig, void *stream) {
    if (n_pairs < 0) return fail(MDM_EINVAL, "negative sample count");
    if (n_pairs == 0) return 0;
    if (!d_raw || !d_sig) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    const int vec = ((uintptr_t)d_raw & 15) == 0 && ((uintptr_t)d_sig & 15) == 0;
    hipLaunchKernelGGL(k_dequantize, grid_for(vec ? (n_pairs + 7) / 8 : n_pairs), dim3(BLOCK), 0, (hipStream_t)stream,
                       d_raw, n_pairs, (float2 *)d_sig, vec);
    return launch_check("k_dequantize");
}

int mdm_iq_dequantize(int device, const uint8_t *raw, long n_pairs, float *sig) {
    if (n_pairs < 0) return fail(MDM_EINVAL, "negative sample count");
    if (n_pairs == 0) return 0;
    if (!raw || !sig) return fail(MDM_EINVAL, "null buffer");
    Guard g(device);
    const size_t ib = (size_t)n_pairs * 2, ob = (size_t)n_pairs * 8;
    Stage s;
    int rc;
    if ((rc = s.init()) || (rc = s.alloc(0, ib)) || (rc = s.alloc(1, ob)) || (rc = s.h2d(0, raw, ib))) return rc;
    if ((rc = mdm_iq_dequantize_dev(device, (const uint8_t *)s.p[0], n_pairs, (float *)s.p[1], s.st))) return rc;
    if ((rc = s.d2h(sig, 1, ob))) return rc;
    return s.sync();
}

}  // extern "C"
