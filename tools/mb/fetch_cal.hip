// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths the
// decoder uses (MI355X_MICROARCH.md: "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").  Each kernel
// moves exactly BYTES bytes of a buffer far larger than the 256 MiB Infinity
// Cache, coalesced, at 16 / 8 / 4 B per lane; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_cal      and      --pmc WRITE_SIZE
// and divide the counter (KiB) by BYTES / 1024.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t BYTES = 2ull << 30;

template <class T>
__global__ void k_read(const T *__restrict__ p, size_t n, float *out) {
    float acc = 0.0f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const T v = p[i];
        acc += reinterpret_cast<const float *>(&v)[0];
    }
    if (acc == 12345.678f) out[0] = acc;   // never true: keeps the loads
}

template <class T>
__global__ void k_write(T *__restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T v;
        reinterpret_cast<float *>(&v)[0] = (float)i;
        for (unsigned j = 1; j < sizeof(T) / 4; ++j) reinterpret_cast<float *>(&v)[j] = 0.0f;
        p[i] = v;
    }
}

int main() {
    void *buf;
    float *out;
    if (hipMalloc(&buf, BYTES) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    hipMemset(buf, 0, BYTES);
    const dim3 g(256 * 32), b(256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto t = [&](const char *name, auto launch) {
        launch();
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s %8.3f ms  %7.1f GB/s\n", name, ms, BYTES / (ms * 1e-3) / 1e9);
    };
    t("read16", [&] { hipLaunchKernelGGL(k_read<float4>, g, b, 0, 0, (const float4 *)buf, BYTES / 16, out); });
    t("read8", [&] { hipLaunchKernelGGL(k_read<float2>, g, b, 0, 0, (const float2 *)buf, BYTES / 8, out); });
    t("read4", [&] { hipLaunchKernelGGL(k_read<float>, g, b, 0, 0, (const float *)buf, BYTES / 4, out); });
    t("write16", [&] { hipLaunchKernelGGL(k_write<float4>, g, b, 0, 0, (float4 *)buf, BYTES / 16); });
    t("write8", [&] { hipLaunchKernelGGL(k_write<float2>, g, b, 0, 0, (float2 *)buf, BYTES / 8); });
    t("write4", [&] { hipLaunchKernelGGL(k_write<float>, g, b, 0, 0, (float *)buf, BYTES / 4); });
    hipDeviceSynchronize();
    printf("bytes per launch: %zu (%.0f KiB)\n", BYTES, BYTES / 1024.0);
    return 0;
}
