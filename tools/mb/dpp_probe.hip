// dpp_probe.hip -- gfx950 DPP semantics and recursion-step latency probe.
//
// 1. For each DPP control used by the frame decoder (tdec_frame.hip) prints the
//    source lane every destination lane of a 16-lane row reads, so the lane ^ x
//    exchanges (x = 8, 4, 2, 1) are checked on the hardware, not assumed.
// 2. Times one wave running a serial max-plus recursion step (partner exchange,
//    two adds, max3, state-0 broadcast, subtract) for 4096 steps, with the
//    partner exchange done by DPP (the frame decoder's form) and by ds_bpermute
//    (the round-3 low-latency decoder's form): cycles per step.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CTL, int BANK>
__device__ __forceinline__ int dpp_upd(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTL, 0xF, BANK, false);
}

__global__ void k_map(int *out) {
    const int l = threadIdx.x;
    out[0 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x128, 0xF, 0xF, false);   // row_ror:8
    out[1 * 64 + l] = dpp_upd<0x114, 0xA>(dpp_upd<0x104, 0x5>(-1, l), l);     // row_shl:4 banks 0,2; row_shr:4 banks 1,3
    out[2 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x4E, 0xF, 0xF, false);    // quad_perm [2,3,0,1]
    out[3 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0xB1, 0xF, 0xF, false);    // quad_perm [1,0,3,2]
    out[4 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x150, 0xF, 0xF, false);   // row_newbcast:0
    out[5 * 64 + l] = __builtin_amdgcn_mov_dpp(l, 0x104, 0xF, 0xF, false);   // row_shl:4 all banks
}

template <int X> __device__ __forceinline__ float xr(float v) {
    const int i = __float_as_int(v);
    if constexpr (X == 8) return __int_as_float(__builtin_amdgcn_mov_dpp(i, 0x128, 0xF, 0xF, false));
    if constexpr (X == 4) return __int_as_float(dpp_upd<0x114, 0xA>(dpp_upd<0x104, 0x5>(i, i), i));
    if constexpr (X == 2) return __int_as_float(__builtin_amdgcn_mov_dpp(i, 0x4E, 0xF, 0xF, false));
    return __int_as_float(__builtin_amdgcn_mov_dpp(i, 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float bc0(float n) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(n), 0x150, 0xF, 0xF, false));
}
template <int X> __device__ __forceinline__ float stepd(float v, float pa, float pb) {
    const float o = xr<X>(v);
    const float n = fmaxf(fmaxf(-1e9f, v + pa), o + pb);
    return n - bc0(n);
}

__global__ void k_time(float *out, long long *cyc, int mode) {
    const int l = threadIdx.x;
    float v = 0.01f * l, pa = 0.3f * (l & 3), pb = -0.2f * (l & 5);
    const long long t0 = clock64();
    if (mode == 0) {
        for (int t = 0; t < 4096; t += 4) {
            v = stepd<8>(v, pa, pb);
            v = stepd<4>(v, pb, pa);
            v = stepd<2>(v, pa, pb);
            v = stepd<1>(v, pb, pa);
        }
    } else {
        const int s0 = (l & ~15) | ((l & 15) >> 1), s1 = s0 | 8;
        for (int t = 0; t < 4096; ++t) {
            const float x = __shfl(v, s0) + pa, y = __shfl(v, s1) + pb;
            const float n = fmaxf(fmaxf(-1e9f, x), y);
            v = n - bc0(n);
        }
    }
    const long long t1 = clock64();
    out[l] = v;
    if (l == 0) cyc[mode] = t1 - t0;
}

int main() {
    int *d;
    hipMalloc(&d, 6 * 64 * sizeof(int));
    hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, d);
    int h[6 * 64];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char *nm[6] = {"row_ror:8", "xor4 (shl4 b0101 | shr4 b1010)", "quad_perm[2,3,0,1]", "quad_perm[1,0,3,2]",
                         "row_newbcast:0", "row_shl:4 all banks"};
    for (int c = 0; c < 6; ++c) {
        printf("%-32s:", nm[c]);
        for (int l = 0; l < 16; ++l) printf(" %d", h[c * 64 + l]);
        printf("  | row1 lane16..19: %d %d %d %d\n", h[c * 64 + 16], h[c * 64 + 17], h[c * 64 + 18], h[c * 64 + 19]);
    }
    float *o;
    long long *cy;
    hipMalloc(&o, 64 * sizeof(float));
    hipMalloc(&cy, 2 * sizeof(long long));
    for (int rep = 0; rep < 2; ++rep)
        for (int m = 0; m < 2; ++m) hipLaunchKernelGGL(k_time, dim3(1), dim3(64), 0, 0, o, cy, m);
    long long c[2];
    hipMemcpy(c, cy, sizeof c, hipMemcpyDeviceToHost);
    printf("cycles per recursion step (clock64): dpp %.1f  ds_bpermute %.1f\n", c[0] / 4096.0, c[1] / 4096.0);
    return 0;
}
