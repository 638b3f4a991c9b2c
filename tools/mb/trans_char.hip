// Characterise gfx950's v_exp_f32 (2^x) and v_log_f32 (log2 x) against the
// correctly rounded results, exhaustively over the domains a build-defined
// log-MAP would feed them: every f32 x in [-64, 0] for 2^x and every f32 in
// [1, 2] for log2.  The reference value is the f64 result (ocml exp2 / log2,
// < 1 ulp of f64) rounded to f32; inputs whose f64 value lies within 8 f64 ulps
// of an f32 rounding midpoint are counted as ambiguous (the f64 reference can
// not decide them) and listed.  Output: counts, and the first mismatches.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct Cnt {
    unsigned long long total, equal, up1, down1, far, amb;
};
constexpr int MAXLIST = 4096;

__device__ __forceinline__ float hw(int which, float x) {
    return which == 0 ? __builtin_amdgcn_exp2f(x) : __builtin_amdgcn_logf(x);
}

__global__ void k_char(int which, uint32_t lo, uint32_t n, Cnt *c, uint32_t *list, unsigned *nlist) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long eq = 0, up = 0, dn = 0, far = 0, amb = 0, tot = 0;
    for (; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t u = lo + i;
        const float x = __uint_as_float(u);
        const float h = hw(which, x);
        const double r = which == 0 ? exp2((double)x) : log2((double)x);
        const float rf = (float)r;
        // ambiguity: distance of r to the f32 midpoint on its side
        const float nb = r >= (double)rf ? nextafterf(rf, INFINITY) : nextafterf(rf, -INFINITY);
        const double mid = 0.5 * ((double)rf + (double)nb);
        const double du = fabs(r) * 0x1p-52;
        const bool am = fabs(r - mid) <= 8.0 * du;
        ++tot;
        const int32_t dh = (int32_t)__float_as_uint(h) - (int32_t)__float_as_uint(rf);
        bool bad = false;
        if (am) {
            ++amb;
            bad = true;
        } else if (h == rf && __float_as_uint(h) == __float_as_uint(rf)) {
            ++eq;
        } else if (dh == 1) {
            ++up;
            bad = true;
        } else if (dh == -1) {
            ++dn;
            bad = true;
        } else {
            ++far;
            bad = true;
        }
        if (bad) {
            const unsigned k = atomicAdd(nlist, 1u);
            if (k < MAXLIST) {
                list[3 * k] = u;
                list[3 * k + 1] = __float_as_uint(h);
                list[3 * k + 2] = __float_as_uint(rf) | (am ? 0 : 0);
            }
        }
    }
    atomicAdd(&c->total, tot);
    atomicAdd(&c->equal, eq);
    atomicAdd(&c->up1, up);
    atomicAdd(&c->down1, dn);
    atomicAdd(&c->far, far);
    atomicAdd(&c->amb, amb);
}

static void run(int which, uint32_t lo, uint32_t hi, const char *name) {
    Cnt *c;
    uint32_t *list;
    unsigned *nl;
    hipMalloc(&c, sizeof(Cnt));
    hipMalloc(&list, 3 * MAXLIST * 4);
    hipMalloc(&nl, 4);
    hipMemset(c, 0, sizeof(Cnt));
    hipMemset(nl, 0, 4);
    const uint32_t n = hi - lo + 1;
    k_char<<<8192, 256>>>(which, lo, n, c, list, nl);
    hipDeviceSynchronize();
    Cnt h;
    unsigned nh;
    static uint32_t hl[3 * MAXLIST];
    hipMemcpy(&h, c, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(&nh, nl, 4, hipMemcpyDeviceToHost);
    hipMemcpy(hl, list, sizeof hl, hipMemcpyDeviceToHost);
    printf("%s [0x%08x, 0x%08x]: total %llu equal %llu +1ulp %llu -1ulp %llu far %llu ambiguous %llu\n", name, lo, hi,
           h.total, h.equal, h.up1, h.down1, h.far, h.amb);
    const unsigned show = nh < 40 ? nh : 40;
    for (unsigned k = 0; k < show; ++k) {
        float x, a, b;
        memcpy(&x, &hl[3 * k], 4);
        memcpy(&a, &hl[3 * k + 1], 4);
        memcpy(&b, &hl[3 * k + 2], 4);
        printf("  x=%a (0x%08x) hw=%a ref=%a\n", x, hl[3 * k], a, b);
    }
    hipFree(c);
    hipFree(list);
    hipFree(nl);
}

int main() {
    // 2^x, x in [-64, -0]: bit patterns 0x80000000 (-0) .. 0xC2800000 (-64)
    run(0, 0x80000000u, 0xC2800000u, "v_exp_f32 x in [-64, 0]");
    // 2^x, x in [0, 1): 0x00000000 .. 0x3F7FFFFF
    run(0, 0x00000000u, 0x3F7FFFFFu, "v_exp_f32 x in [0, 1)");
    // log2 x, x in [1, 2]: 0x3F800000 .. 0x40000000
    run(1, 0x3F800000u, 0x40000000u, "v_log_f32 x in [1, 2]");
    // log2 x, x in [0.5, 1)
    run(1, 0x3F000000u, 0x3F7FFFFFu, "v_log_f32 x in [0.5, 1)");
    return 0;
}
