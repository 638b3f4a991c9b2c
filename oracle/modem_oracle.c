/*
 * modem_oracle.c -- CPU restatement of the reference's modem front-end
 * (SURVEY.md §8(f) row 4).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker of libmodem.so.  Only tests/
 * load it (through oracle/oracle.py); the product path never does.
 *
 *   orm_map             the mappers: sdr_modem.py:101-207, modulators.py:119-197,
 *                       test_sdr_with_coding.py:25-86 (label MSB first, zero pad,
 *                       table lookup; tables are the reference's values)
 *   orm_demod_gt0       sdr_modem.py:104-105, modulators.py:121-122
 *   orm_demod_qpsk      sdr_modem.py:114-118, modulators.py:133-136
 *   orm_demod_psk8_*    sdr_modem.py:132-140 (per-symbol loop: int(NaN) raises),
 *                       modulators.py:147-155 (array: astype(int) of NaN -> 0 after % 8)
 *   orm_demod_qam_axis  sdr_modem.py:156-220 (f64: x * np.sqrt(S), round half even, clip)
 *   orm_demod_argmin    modulators.py:165-171 (np.argmin of numpy's complex128 |s - c|)
 *   orm_fir             np.convolve 'same' of sdr_modem.py:93-97, scipy upfirdn of
 *                       modulators.py:67-83, full convolution + [2d::sps] of :85-113,
 *                       by definition (sum over taps in ascending order; the
 *                       reference's BLAS / scipy summation order is not defined,
 *                       so FIR parity is a tolerance)
 *   orm_iq_quantize_*   sdr_modem.py:329-335 (numpy's complex division -- Smith's
 *                       method -- and complex product in the signal's precision,
 *                       * 127, clip, C cast to int8; NaN -> 0 as numpy on x86)
 *   orm_iq_dequantize   sdr_modem.py:337-342
 *
 * Strict IEEE (-ffp-contract=off); fma only where numpy's own loop fuses (|z|).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------------ mappers -- */
void orm_map(const uint8_t *bits, long n_bits, int bps, const double *table, double *out)
{
    long n_sym = (n_bits + bps - 1) / bps;
    for (long s = 0; s < n_sym; ++s) {
        int lab = 0;
        for (int j = 0; j < bps; ++j) {
            long q = s * bps + j;
            lab = lab * 2 + (q < n_bits ? bits[q] : 0);
        }
        out[2 * s] = table[2 * lab];
        out[2 * s + 1] = table[2 * lab + 1];
    }
}

/* ------------------------------------------------------------------ demods --- */
static void put_bits(uint8_t *o, int v, int n)
{
    for (int b = 0; b < n; ++b) o[b] = (uint8_t)((v >> (n - 1 - b)) & 1);
}

void orm_demod_gt0(const double *syms, long n, uint8_t *bits)
{
    for (long s = 0; s < n; ++s) bits[s] = syms[2 * s] > 0.0;
}

void orm_demod_qpsk(const double *syms, long n, uint8_t *bits)
{
    for (long s = 0; s < n; ++s) {
        bits[2 * s] = syms[2 * s] < 0.0;
        bits[2 * s + 1] = syms[2 * s + 1] < 0.0;
    }
}

/* phase = np.angle(s); if phase < 0: phase += 2*np.pi; idx = int(np.round(phase / (np.pi/4))) % 8
 * -- numpy scalars of the symbols' dtype absorb the Python floats (NEP 50). */
long orm_demod_psk8_f32(const float *syms, long n, const int *labels, int nan_raises, uint8_t *bits)
{
    long nans = 0;
    for (long s = 0; s < n; ++s) {
        float ph = atan2f(syms[2 * s + 1], syms[2 * s]);
        if (ph < 0.0f) ph += (float)(2.0 * M_PI);
        float q = rintf(ph / (float)(M_PI / 4.0));
        int idx = 0;
        if (isnan(q)) nans += nan_raises;
        else idx = ((int)q) % 8;
        put_bits(bits + 3 * s, labels[idx], 3);
    }
    return nans;
}

long orm_demod_psk8_f64(const double *syms, long n, const int *labels, int nan_raises, uint8_t *bits)
{
    long nans = 0;
    for (long s = 0; s < n; ++s) {
        double ph = atan2(syms[2 * s + 1], syms[2 * s]);
        if (ph < 0.0) ph += 2.0 * M_PI;
        double q = rint(ph / (M_PI / 4.0));
        int idx = 0;
        if (isnan(q)) nans += nan_raises;
        else idx = ((int)q) % 8;
        put_bits(bits + 3 * s, labels[idx], 3);
    }
    return nans;
}

/* I = np.real(s) * np.sqrt(S) (float64); i_idx = int(np.clip(np.round((I + L-1) / 2), 0, L-1)) */
long orm_demod_qam_axis(const double *syms, long n, int k, double scale, const int *labels, uint8_t *bits)
{
    long nans = 0;
    int L = 1 << k;
    for (long s = 0; s < n; ++s) {
        for (int ax = 0; ax < 2; ++ax) {
            double x = syms[2 * s + ax] * scale;
            double q = rint((x + (double)(L - 1)) / 2.0);
            int idx = 0;
            if (isnan(q)) ++nans;
            else {
                if (q < 0.0) q = 0.0;
                if (q > (double)(L - 1)) q = (double)(L - 1);
                idx = (int)q;
            }
            put_bits(bits + 2 * k * s + k * ax, labels[idx], k);
        }
    }
    return nans;
}

static double cabs_np_f64(double re, double im) /* numpy's complex |z| (SIMD loop, FMA host) */
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
    return sqrt(fma(ratio, ratio, 1.0)) * larger;
}

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
    return sqrtf(fmaf(ratio, ratio, 1.0f)) * larger;
}

/* idxs = np.argmin(np.abs(symbols[:, None] - c[None, :]), axis=1): first minimum, NaN first */
void orm_demod_argmin(const double *syms, long n, int bps, const double *cons, uint8_t *bits)
{
    int M = 1 << bps;
    for (long s = 0; s < n; ++s) {
        int idx = -1;
        double best = 0.0;
        for (int m = 0; m < M; ++m) {
            double d = cabs_np_f64(syms[2 * s] - cons[2 * m], syms[2 * s + 1] - cons[2 * m + 1]);
            if (idx < 0 || isnan(d) || d < best) {
                idx = m;
                best = d;
                if (isnan(d)) break;
            }
        }
        put_bits(bits + (long)bps * s, idx, bps);
    }
}

/* ------------------------------------------------------------------ FIR ------ */
/* out[i] = sum_{k} h[k] * xu[i*down + off - k], xu the up-sampled input (zeros between samples) */
void orm_fir(const double *x, long n_x, const double *h, int L, int up, int down, long off, long n_out, double *out)
{
    for (long i = 0; i < n_out; ++i) {
        long j = i * down + off;
        double re = 0.0, im = 0.0;
        for (int k = 0; k < L; ++k) {
            long q = j - k;
            if (q < 0 || q % up) continue;
            long m = q / up;
            if (m >= n_x) continue;
            re += h[k] * x[2 * m];
            im += h[k] * x[2 * m + 1];
        }
        out[2 * i] = re;
        out[2 * i + 1] = im;
    }
}

/* ------------------------------------------------------------------ IQ ------- */
/* numpy complex division (loops.c.src, Smith's method) and product */
#define CDIV(T, FABS, ar, ai, br, bi, qr, qi)                                   \
    do {                                                                        \
        T abr = FABS(br), abi = FABS(bi);                                       \
        if (abr >= abi) {                                                       \
            if (abr == 0 && abi == 0) { qr = ar / abr; qi = ai / abr; }        \
            else {                                                              \
                T rat = bi / br, scl = (T)1 / (br + bi * rat);                  \
                qr = (ar + ai * rat) * scl; qi = (ai - ar * rat) * scl;         \
            }                                                                   \
        } else {                                                                \
            T rat = br / bi, scl = (T)1 / (bi + br * rat);                      \
            qr = (ar * rat + ai) * scl; qi = (ai * rat - ar) * scl;             \
        }                                                                       \
    } while (0)

static int8_t i8_f64(double v)
{
    v = v * 127.0;
    if (v != v) return 0;
    if (v < -127.0) v = -127.0;
    if (v > 127.0) v = 127.0;
    return (int8_t)(int)v;
}

static int8_t i8_f32(float v)
{
    v = v * 127.0f;
    if (v != v) return 0;
    if (v < -127.0f) v = -127.0f;
    if (v > 127.0f) v = 127.0f;
    return (int8_t)(int)v;
}

void orm_iq_quantize_f64(const double *sig, long n, int8_t *out)
{
    double mx = 0.0;
    int nan = 0;
    for (long i = 0; i < n; ++i) {
        double a = cabs_np_f64(sig[2 * i], sig[2 * i + 1]);
        if (a != a) nan = 1;
        else if (a > mx) mx = a;
    }
    double d = (nan ? NAN : mx) + 1e-10;
    for (long i = 0; i < n; ++i) {
        double qr, qi;
        CDIV(double, fabs, sig[2 * i], sig[2 * i + 1], d, 0.0, qr, qi);
        double pr = qr * 0.95 - qi * 0.0, pi = qr * 0.0 + qi * 0.95;
        out[2 * i] = i8_f64(pr);
        out[2 * i + 1] = i8_f64(pi);
    }
}

void orm_iq_quantize_f32(const float *sig, long n, int8_t *out)
{
    float mx = 0.0f;
    int nan = 0;
    for (long i = 0; i < n; ++i) {
        float a = cabs_np_f32(sig[2 * i], sig[2 * i + 1]);
        if (a != a) nan = 1;
        else if (a > mx) mx = a;
    }
    float d = (nan ? NAN : mx) + (float)1e-10;
    for (long i = 0; i < n; ++i) {
        float qr, qi;
        CDIV(float, fabsf, sig[2 * i], sig[2 * i + 1], d, 0.0f, qr, qi);
        float pr = qr * 0.95f - qi * 0.0f, pi = qr * 0.0f + qi * 0.95f;
        out[2 * i] = i8_f32(pr);
        out[2 * i + 1] = i8_f32(pi);
    }
}

void orm_iq_dequantize(const uint8_t *raw, long n_pairs, float *out)
{
    for (long i = 0; i < n_pairs; ++i) {
        out[2 * i] = ((float)raw[2 * i] - 127.5f) / 127.5f;
        out[2 * i + 1] = ((float)raw[2 * i + 1] - 127.5f) / 127.5f;
    }
}
