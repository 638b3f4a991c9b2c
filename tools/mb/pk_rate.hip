// Micro-benchmark: issue rate of v_pk_add_f32 vs v_add_f32 (8 independent chains).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
template <int PK> __global__ __launch_bounds__(256) void k(float *out, int iters, float d) {
    float x[16];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            if (PK) {
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    f2 v = f2{x[i], x[i + 1]};
                    asm volatile("v_pk_add_f32 %0, %0, %1 op_sel_hi:[1,0]" : "+v"(v) : "v"(f2{d, d}));
                    x[i] = v.x; x[i + 1] = v.y;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[i]) : "v"(d));
            }
        }
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    float *o;
    hipMalloc(&o, 4 << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 20000;
    for (int occ = 1; occ <= 2; ++occ) {
        int blocks = 256 * occ;   // 256 CUs x (4 waves x occ) -> occ waves per SIMD
        for (int pk = 0; pk < 2; ++pk) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                if (pk) k<1><<<blocks, 256>>>(o, iters, 1e-7f); else k<0><<<blocks, 256>>>(o, iters, 1e-7f);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                double lane_adds = (double)blocks * 256 * iters * 8 * 16;
                double instrs = lane_adds / (pk ? 2 : 1) / 64;   // wave instructions
                if (rep) printf("waves/SIMD %d %s: %.3f ms  %.1f T lane-adds/s  %.2f cyc/wave-instr/SIMD @2.4GHz\n", occ,
                                pk ? "v_pk_add_f32" : "v_add_f32  ", ms, lane_adds / ms / 1e9,
                                (ms * 1e-3 * 2.4e9) / (instrs / 1024));
            }
        }
    }
    return 0;
}
