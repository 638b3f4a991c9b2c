// Mixed read/write streaming bandwidth at 16-B vs 8-B per lane (decoder-like: 2 reads per write),
// to see whether splitting the decoder's 16-B stores into 8-B planes would help.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = 1ull << 30;   // per buffer

template <class T>
__global__ void k_mix(const T *__restrict__ a, const T *__restrict__ b, T *__restrict__ c, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T x = a[i], y = b[i], z;
        for (unsigned j = 0; j < sizeof(T) / 4; ++j)
            reinterpret_cast<float *>(&z)[j] = reinterpret_cast<float *>(&x)[j] + reinterpret_cast<float *>(&y)[j];
        c[i] = z;
    }
}

int main() {
    void *a, *b, *c;
    if (hipMalloc(&a, BYTES) || hipMalloc(&b, BYTES) || hipMalloc(&c, BYTES)) return 1;
    hipMemset(a, 0, BYTES);
    hipMemset(b, 0, BYTES);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto t = [&](const char *name, auto launch) {
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 4; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 4;
        printf("%-12s %8.3f ms  %7.1f GB/s (2 reads + 1 write of 1 GiB)\n", name, ms, 3.0 * BYTES / (ms * 1e-3) / 1e9);
    };
    for (int g : {2048, 8192, 32768}) {
        printf("grid %d x 256\n", g);
        t("mix16", [&] { hipLaunchKernelGGL(k_mix<float4>, dim3(g), dim3(256), 0, 0, (const float4 *)a, (const float4 *)b, (float4 *)c, BYTES / 16); });
        t("mix8", [&] { hipLaunchKernelGGL(k_mix<float2>, dim3(g), dim3(256), 0, 0, (const float2 *)a, (const float2 *)b, (float2 *)c, BYTES / 8); });
        t("mix4", [&] { hipLaunchKernelGGL(k_mix<float>, dim3(g), dim3(256), 0, 0, (const float *)a, (const float *)b, (float *)c, BYTES / 4); });
    }
    return 0;
}
