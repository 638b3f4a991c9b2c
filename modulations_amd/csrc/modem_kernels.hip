// modem_kernels.hip -- gfx950 kernels of the modem front-end (SURVEY.md §8(f)
// row 4): mappers, hard demodulators, polyphase FIR, IQ sample conversion.
//
// All of these are byte-moving elementwise passes (HBM-bound): one thread per
// output element, grid-stride, tables staged once per block in LDS, the FIR's
// input window staged in LDS so every input sample is fetched from HBM once
// per block.  Arithmetic restates the reference's numpy expressions in the
// precision numpy uses for them (npmath.hip); the build keeps IEEE denormals
// and no FMA contraction (-ffp-contract=off), explicit fma() only where
// numpy's own loop fuses (|z|) or where the reference's sum order is not
// defined (the FIR: BLAS / scipy order, compared within a tolerance).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "npmath.hip"

namespace mdm {

constexpr int BLOCK = 256;
constexpr int MAP_MAX = 256;    // points of a mapper table (f32; 128 for f64)
constexpr int TAPS_MAX = 256;   // FIR taps
constexpr int ARG_MAX = 64;     // points of an argmin table

__device__ __forceinline__ long gtid() { return (long)blockIdx.x * BLOCK + threadIdx.x; }
__device__ __forceinline__ long gstride() { return (long)gridDim.x * BLOCK; }

// ---- mapper: bits (MSB-first labels, zero padded) -> table[label] ---------------------
struct MapTable {
    union {
        float f[2 * MAP_MAX];
        double d[MAP_MAX];   // MAP_MAX/2 complex128 points
    };
};

template <typename T> struct C2;
template <> struct C2<float> { typedef float2 t; };
template <> struct C2<double> { typedef double2 t; };

template <typename T>
__global__ __launch_bounds__(BLOCK) void k_map(const uint8_t *__restrict__ bits, long n_bits, int bps, long n_sym,
                                               MapTable tab, typename C2<T>::t *__restrict__ out) {
    typedef typename C2<T>::t V;
    __shared__ V t[MAP_MAX];
    const T *src = sizeof(T) == 4 ? (const T *)tab.f : (const T *)tab.d;
    for (int i = threadIdx.x; i < (1 << bps); i += BLOCK) {
        V v;
        v.x = src[2 * i];
        v.y = src[2 * i + 1];
        t[i] = v;
    }
    __syncthreads();
    for (long s = gtid(); s < n_sym; s += gstride()) {
        const long b0 = s * bps;
        int lab = 0;
        if (b0 + bps <= n_bits) {
            for (int j = 0; j < bps; ++j) lab = (lab << 1) | (bits[b0 + j] & 1);
        } else {
            for (int j = 0; j < bps; ++j) lab = (lab << 1) | (b0 + j < n_bits ? (bits[b0 + j] & 1) : 0);
        }
        out[s] = t[lab];
    }
}

// ---- hard demodulators -------------------------------------------------------------------
struct DemodArgs {
    int kind, bps, nan_raises, levels;
    double scale;
    int32_t labels[256];
    double cons[2 * ARG_MAX];
};

// round(angle / (pi/4)) of the 8PSK demods in the symbols' precision:
// np.angle -> arctan2; `if phase < 0: phase += 2*np.pi` (a Python float added
// to a numpy scalar of the symbols' dtype stays in that dtype); / (np.pi/4);
// np.round = round half to even.
template <typename T> __device__ __forceinline__ T psk8_sector(T re, T im) {
    T ph = atan2(im, re);
    if (ph < (T)0) ph = ph + (T)6.283185307179586;
    return rint(ph / (T)0.7853981633974483);
}

template <typename T>
__global__ __launch_bounds__(BLOCK) void k_demod(const typename C2<T>::t *__restrict__ syms, long n_sym, DemodArgs a,
                                                 uint8_t *__restrict__ bits, uint32_t *__restrict__ nan_count) {
    __shared__ int lab[256];
    __shared__ double cons[2 * ARG_MAX];
    for (int i = threadIdx.x; i < 256; i += BLOCK) lab[i] = a.labels[i];
    for (int i = threadIdx.x; i < 2 * ARG_MAX; i += BLOCK) cons[i] = a.cons[i];
    __syncthreads();
    uint32_t nans = 0;
    for (long s = gtid(); s < n_sym; s += gstride()) {
        const T re = syms[s].x, im = syms[s].y;
        uint8_t *o = bits + s * a.bps;
        if (a.kind == 0) {                      // MDM_DEMOD_GT0
            o[0] = re > (T)0;
        } else if (a.kind == 1) {               // MDM_DEMOD_QPSK
            o[0] = re < (T)0;
            o[1] = im < (T)0;
        } else if (a.kind == 2) {               // MDM_DEMOD_PSK8
            const T r = psk8_sector<T>(re, im);
            int idx = 0;
            if (r != r) nans += a.nan_raises;   // int(NaN) raises; astype(int) -> INT64_MIN, % 8 = 0
            else idx = ((int)r) & 7;            // r in [0, 8]
            const int l = lab[idx];
            o[0] = (l >> 2) & 1;
            o[1] = (l >> 1) & 1;
            o[2] = l & 1;
        } else if (a.kind == 3) {               // MDM_DEMOD_QAM_AXIS (f64, np.float64 scale)
            const int K = a.bps / 2, L = a.levels;
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {
                const double x = (double)(ax ? im : re) * a.scale;
                double q = rint((x + (double)(L - 1)) / 2.0);
                int idx = 0;
                if (q != q) nans += 1;          // int(np.clip(np.round(NaN))) raises
                else {
                    q = q < 0.0 ? 0.0 : (q > (double)(L - 1) ? (double)(L - 1) : q);
                    idx = (int)q;
                }
                const int l = lab[idx];
                for (int b = 0; b < K; ++b) o[ax * K + b] = (l >> (K - 1 - b)) & 1;
            }
        } else {                                // MDM_DEMOD_ARGMIN: first index of the minimum, NaN wins
            const int M = 1 << a.bps;
            const double sr = (double)re, si = (double)im;
            int idx = 0;
            double best = npm::cabs_np<double>(sr - cons[0], si - cons[1]);
            for (int m = 1; m < M; ++m) {
                if (best != best) break;
                const double d = npm::cabs_np<double>(sr - cons[2 * m], si - cons[2 * m + 1]);
                if (d < best || d != d) {
                    best = d;
                    idx = m;
                }
            }
            for (int b = 0; b < a.bps; ++b) o[b] = (idx >> (a.bps - 1 - b)) & 1;
        }
    }
    if (nan_count && nans) atomicAdd(nan_count, nans);
}

// ---- polyphase up-sample / FIR / down-sample ------------------------------------------
//   out[i] = sum_k h[k] * xu[i*down + off - k],  xu[j] = x[j/up] (j % up == 0, in range) else 0
// One block = FIR_OPB consecutive outputs; the input samples they touch are
// staged once in LDS (as f64) when they fit, else read through L1/L2.
struct FirArgs {
    int n_taps, up, down, per_thread;
    long off, n_out, n_x;
    double h[TAPS_MAX];
};
constexpr int FIR_LDS = 3840;   // staged input samples (60 KiB of double2)

__device__ __forceinline__ long fdiv_floor(long a, long b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

template <typename T, bool STAGE>
__global__ __launch_bounds__(BLOCK) void k_fir(const typename C2<T>::t *__restrict__ x, FirArgs a,
                                               double2 *__restrict__ out) {
    __shared__ double h[TAPS_MAX];
    __shared__ double2 xs[STAGE ? FIR_LDS : 1];
    for (int i = threadIdx.x; i < a.n_taps; i += BLOCK) h[i] = a.h[i];
    const long opb = (long)BLOCK * a.per_thread;
    const long i0 = (long)blockIdx.x * opb;
    // input samples of this block's outputs: m in [m_lo, m_hi]
    const long j_lo = i0 * a.down + a.off - (a.n_taps - 1);
    const long j_hi = (i0 + opb - 1) * a.down + a.off;
    long m_lo = -fdiv_floor(-j_lo, a.up);   // ceil(j_lo / up)
    long m_hi = fdiv_floor(j_hi, a.up);
    m_lo = m_lo < 0 ? 0 : m_lo;
    m_hi = m_hi > a.n_x - 1 ? a.n_x - 1 : m_hi;
    if (STAGE) {
        for (long m = m_lo + threadIdx.x; m <= m_hi; m += BLOCK) {
            const typename C2<T>::t v = x[m];
            xs[m - m_lo] = make_double2((double)v.x, (double)v.y);
        }
    }
    __syncthreads();
    for (int r = 0; r < a.per_thread; ++r) {
        const long i = i0 + (long)r * BLOCK + threadIdx.x;
        if (i >= a.n_out) break;
        const long j0 = i * a.down + a.off;
        // taps k with (j0 - k) % up == 0 and 0 <= (j0 - k) / up < n_x
        long kmin = j0 - (a.n_x - 1) * a.up;
        kmin = kmin < 0 ? 0 : kmin;
        const long kmax = j0 < a.n_taps - 1 ? j0 : a.n_taps - 1;
        long k = kmin + ((j0 - kmin) % a.up);
        double re = 0.0, im = 0.0;
        for (; k <= kmax; k += a.up) {
            const long m = (j0 - k) / a.up;
            double xr, xi;
            if (STAGE) {
                const double2 v = xs[m - m_lo];
                xr = v.x;
                xi = v.y;
            } else {
                const typename C2<T>::t v = x[m];
                xr = (double)v.x;
                xi = (double)v.y;
            }
            re = fma(h[k], xr, re);
            im = fma(h[k], xi, im);
        }
        out[i] = make_double2(re, im);
    }
}

// ---- IQ sample conversion ------------------------------------------------------------------
// max|sig| (np.max(np.abs(sig)), NaN propagating) as the largest bit pattern:
// abs values are >= +0, so their IEEE bits order like unsigned integers and a
// NaN outranks +inf.
template <typename T>
__global__ __launch_bounds__(BLOCK) void k_absmax(const typename C2<T>::t *__restrict__ sig, long n,
                                                  unsigned long long *__restrict__ mx) {
    unsigned long long m = 0;
    for (long i = gtid(); i < n; i += gstride()) {
        const T a = npm::cabs_np<T>(sig[i].x, sig[i].y);
        unsigned long long b;
        if (sizeof(T) == 8) b = (unsigned long long)__double_as_longlong((double)a);
        else b = (unsigned long long)(unsigned)__float_as_uint((float)a);
        m = b > m ? b : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(m, o, 64);
        m = v > m ? v : m;
    }
    if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}

template <typename T> __device__ __forceinline__ int8_t to_i8(T v) {
    v = v * (T)127;                                           // np.real(sig) * 127
    if (v != v) return 0;                                     // astype(int8) of NaN (x86 numpy)
    v = v < (T)-127 ? (T)-127 : (v > (T)127 ? (T)127 : v);    // np.clip
    return (int8_t)(int)v;                                    // C cast: truncation toward zero
}

template <typename T>
__global__ __launch_bounds__(BLOCK) void k_quantize(const typename C2<T>::t *__restrict__ sig, long n,
                                                    const unsigned long long *__restrict__ mx,
                                                    char2 *__restrict__ iq) {
    T amax;
    if (sizeof(T) == 8) amax = (T)__longlong_as_double((long long)*mx);
    else amax = (T)__uint_as_float((unsigned)*mx);
    const T d = amax + (T)1e-10;   // np.max(...) + 1e-10 in the signal's precision
    for (long i = gtid(); i < n; i += gstride()) {
        T qr, qi, pr, pi;
        npm::cdiv_np<T>(sig[i].x, sig[i].y, d, (T)0, qr, qi);       // sig / d (complex division)
        npm::cmul_np<T>(qr, qi, (T)0.95, (T)0, pr, pi);              // * 0.95 (complex product)
        iq[i] = make_char2(to_i8<T>(pr), to_i8<T>(pi));
    }
}

// (raw.astype(np.float32) - 127.5) / 127.5, I from even bytes, Q from odd
__global__ __launch_bounds__(BLOCK) void k_dequantize(const uchar2 *__restrict__ raw, long n, float2 *__restrict__ sig) {
    for (long i = gtid(); i < n; i += gstride()) {
        const uchar2 r = raw[i];
        sig[i] = make_float2(((float)r.x - 127.5f) / 127.5f, ((float)r.y - 127.5f) / 127.5f);
    }
}

}  // namespace mdm
