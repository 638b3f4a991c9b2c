// Throughput of the log-MAP max* forms at two waves per SIMD (the decoder's
// occupancy): 16 independent chains per lane, acc[i] = max*(acc[i], acc[i+1] + c).
//   0: maxNum only (max-log)
//   1: round-2 definition: maxNum + log1p_01(exp_neg(min(|a-b|, 150))) (polynomials)
//   2: base-2 hardware form: maxNum + v_log_f32(1 + v_exp_f32(-|a-b|))
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

__device__ __forceinline__ float exp_neg(float d) {
    const float x = d * 0x1.715476p+0f;
    const int nn = (int)(-x);
    const float f = __builtin_amdgcn_fractf(x);
    float p = -0x1.f0ca8p-11f;
    p = fmaf(p, f, 0x1.2dd26cp-7f);
    p = fmaf(p, f, -0x1.c503aep-5f);
    p = fmaf(p, f, 0x1.ebe33ap-3f);
    p = fmaf(p, f, -0x1.62e3aap-1f);
    p = fmaf(p, f, 0x1.fffffep-1f);
    return ldexpf(p, nn);
}
__device__ __forceinline__ float log1p_01(float e) {
    float q = -0x1.18f998p-7f;
    q = fmaf(q, e, 0x1.6a33e2p-5f);
    q = fmaf(q, e, -0x1.b9c4c8p-4f);
    q = fmaf(q, e, 0x1.6ba9f2p-3f);
    q = fmaf(q, e, -0x1.f5c086p-3f);
    q = fmaf(q, e, 0x1.54bf8p-2f);
    q = fmaf(q, e, -0x1.fff95p-2f);
    q = fmaf(q, e, 0x1.fffffap-1f);
    return q * e;
}
template <int V> __device__ __forceinline__ float mstar(float a, float b) {
    if constexpr (V == 0) return fmaxf(a, b);
    if constexpr (V == 1) return fmaxf(a, b) + log1p_01(exp_neg(fminf(fabsf(a - b), 150.0f)));
    return fmaxf(a, b) + __builtin_amdgcn_logf(1.0f + __builtin_amdgcn_exp2f(-fabsf(a - b)));
}
template <int V> __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k(float *out, int iters, float c) {
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 0.001f + i * 0.37f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) x[i] = mstar<V>(x[i], x[(i + 1) & 15] + c) - c;
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    float *o;
    (void)hipMalloc(&o, 4 << 20);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int iters = 4000, blocks = 512;   // 256 CUs x 8 waves = 2 waves per SIMD
    const char *name[3] = {"maxNum", "poly max* (round 2)", "hw base-2 max*"};
    for (int v = 0; v < 3; ++v) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            if (v == 0) k<0><<<blocks, 256>>>(o, iters, 0.25f);
            if (v == 1) k<1><<<blocks, 256>>>(o, iters, 0.25f);
            if (v == 2) k<2><<<blocks, 256>>>(o, iters, 0.25f);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        const double ops = (double)blocks * 256 * iters * 16;
        printf("%-22s %.3f ms  %.2f G max*/s (lane)  %.3f ns per wave-max* per SIMD\n", name[v], best, ops / best / 1e6,
               best * 1e6 / (ops / 64 / 1024));
    }
    return 0;
}
