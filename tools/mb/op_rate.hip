// Micro-benchmark: issue cost (shader cycles per wave-instruction, per wave) of
// the VALU operations the decoders use, 8 independent chains, at 1 and 2 waves
// per SIMD (blocks of 4 waves, one block / two blocks per CU).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
enum { ADD32, PKADD, MAX3, ADD64, MUL64, CVT64_32, CVT32_64, FMA32, NOPS };
static const char *names[] = {"v_add_f32", "v_pk_add_f32", "v_max3_f32", "v_add_f64", "v_mul_f64",
                              "v_cvt_f32_f64", "v_cvt_f64_f32", "v_fma_f32"};
template <int OP> __global__ __launch_bounds__(256) void k(float *out, unsigned long long *cyc, int iters, float d) {
    float x[16];
    double y[8];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int i = 0; i < 8; ++i) y[i] = threadIdx.x * 0.001 + i;
    const double dd = d;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (OP == ADD32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(d));
                if constexpr (OP == FMA32) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x[i]) : "v"(d));
                if constexpr (OP == MAX3) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x[i]) : "v"(d), "v"(x[i + 8]));
                if constexpr (OP == PKADD) {
                    f2 v = f2{x[i], x[i + 8]};
                    asm volatile("v_pk_add_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(v) : "v"(f2{d, d}));
                    x[i] = v.x; x[i + 8] = v.y;
                }
                if constexpr (OP == ADD64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(y[i]) : "v"(dd));
                if constexpr (OP == MUL64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(y[i]) : "v"(dd));
                if constexpr (OP == CVT64_32) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(x[i]) : "v"(y[i]));
                if constexpr (OP == CVT32_64) asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(y[i]) : "v"(x[i]));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    for (int i = 0; i < 8; ++i) s += (float)y[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}
template <int OP> void run(int n_cu, int per_cu, float *o, unsigned long long *c) {
    const int iters = 2000, blocks = n_cu * per_cu;
    k<OP><<<blocks, 256>>>(o, c, iters, 1e-7f);
    hipDeviceSynchronize();
    k<OP><<<blocks, 256>>>(o, c, iters, 1e-7f);
    hipDeviceSynchronize();
    static unsigned long long h[256 * 8 * 4];
    hipMemcpy(h, c, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < blocks * 4; ++i) m += h[i];
    m /= blocks * 4;
    printf("%-16s waves/SIMD %d: %.2f cycles per wave-instruction (per wave)\n", names[OP], per_cu, m / (iters * 64.0));
}
int main() {
    int n_cu = 0;
    hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    float *o;
    unsigned long long *c;
    hipMalloc(&o, sizeof(float) * 256 * 256 * 8);
    hipMalloc(&c, sizeof(unsigned long long) * 256 * 8 * 4);
    for (int w = 1; w <= 2; ++w) {
        run<ADD32>(n_cu, w, o, c); run<FMA32>(n_cu, w, o, c); run<PKADD>(n_cu, w, o, c); run<MAX3>(n_cu, w, o, c);
        run<ADD64>(n_cu, w, o, c); run<MUL64>(n_cu, w, o, c); run<CVT64_32>(n_cu, w, o, c); run<CVT32_64>(n_cu, w, o, c);
    }
    return 0;
}
