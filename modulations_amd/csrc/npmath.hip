// npmath.hip -- numpy's elementwise arithmetic restated for the gfx950 kernels
// (shared by tdec_kernels.hip and modem_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace npm {

// numpy's complex |z| (the SIMD loop of umath on an FMA host, complex64 and
// complex128 alike): larger * sqrt(fma(r, r, 1)), r = smaller / larger, with
// its inf / NaN handling.
template <typename T> __device__ __forceinline__ T cabs_np(T re, T im) {
    const T inf = (T)INFINITY;
    re = fabs(re);
    im = fabs(im);
    const bool re_inf = re == inf, im_inf = im == inf;
    im = re_inf ? inf : im;
    re = im_inf ? inf : re;
    const bool re_nn = re == re, im_nn = im == im;
    im = re_nn ? im : (T)NAN;
    re = im_nn ? re : (T)NAN;
    const T larger = re > im ? re : im;
    const T smaller = im < re ? im : re;
    const bool div = !(larger == (T)0 || smaller == inf);
    const T ratio = div ? smaller / larger : (T)0;
    const T h = sqrt(fma(ratio, ratio, (T)1));
    return h * larger;
}

// numpy's complex division a / (br + j bi) (Smith's method, loops.c.src).
template <typename T> __device__ __forceinline__ void cdiv_np(T ar, T ai, T br, T bi, T &qr, T &qi) {
    const T abr = fabs(br), abi = fabs(bi);
    if (abr >= abi) {
        if (abr == (T)0 && abi == (T)0) {
            qr = ar / abr;
            qi = ai / abr;
        } else {
            const T rat = bi / br;
            const T scl = (T)1 / (br + bi * rat);
            qr = (ar + ai * rat) * scl;
            qi = (ai - ar * rat) * scl;
        }
    } else {
        const T rat = br / bi;
        const T scl = (T)1 / (bi + br * rat);
        qr = (ar * rat + ai) * scl;
        qi = (ai * rat - ar) * scl;
    }
}

// numpy's complex product (ar + j ai)(br + j bi) = (ar br - ai bi) + j (ar bi + ai br).
template <typename T> __device__ __forceinline__ void cmul_np(T ar, T ai, T br, T bi, T &pr, T &pi) {
    pr = ar * br - ai * bi;
    pi = ar * bi + ai * br;
}

}  // namespace npm
