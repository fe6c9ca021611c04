// stream-copy variants on one MI355X (bench.py's roofline.frac_of_copy needs a copy peak measured
// in the same run; this picks the kernel shape gs_stream_copy_gbs uses)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_one(const float4 *__restrict__ s, float4 *__restrict__ d, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = s[i];
}
__global__ void k_one_nt(const float4 *__restrict__ s, float4 *__restrict__ d, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    typedef float f4 __attribute__((ext_vector_type(4)));
    if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load((const f4 *)&s[i]), (f4 *)&d[i]);
}
template <int U>
__global__ void k_gs(const float4 *__restrict__ s, float4 *__restrict__ d, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) d[i + u * stride] = v[u];
    }
    for (; i < n; i += stride) d[i] = s[i];
}
// each thread a contiguous run of U float4 per step (blocked)
template <int U>
__global__ void k_blk(const float4 *__restrict__ s, float4 *__restrict__ d, size_t n) {
    size_t base = ((size_t)blockIdx.x * blockDim.x) * U + threadIdx.x;
    if (base + (U - 1) * blockDim.x < n) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = s[base + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < U; ++u) d[base + u * blockDim.x] = v[u];
    }
}

int main() {
    const size_t bytes = 1ull << 30, n = bytes / 16;
    float4 *a, *b;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMemset(a, 0, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        std::vector<double> r;
        for (int i = 0; i < 12; ++i) {
            const bool ab = i & 1;
            hipEventRecord(e0);
            launch(ab ? a : b, ab ? b : a);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (i >= 2) r.push_back(2.0 * bytes / (ms * 1e-3) / 1e9);
        }
        std::sort(r.begin(), r.end());
        printf("%-28s median %7.1f GB/s  best %7.1f\n", name, r[r.size() / 2], r.back());
    };
    run("one float4/thread, 256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_one, dim3((n + 255) / 256), dim3(256), 0, 0, s, d, n); });
    run("one float4/thread, 1024", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_one, dim3((n + 1023) / 1024), dim3(1024), 0, 0, s, d, n); });
    run("one float4/thread nt", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_one_nt, dim3((n + 255) / 256), dim3(256), 0, 0, s, d, n); });
    run("grid-stride x4, 2048x256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_gs<4>, dim3(2048), dim3(256), 0, 0, s, d, n); });
    run("grid-stride x4, 8192x256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_gs<4>, dim3(8192), dim3(256), 0, 0, s, d, n); });
    run("grid-stride x8, 4096x256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_gs<8>, dim3(4096), dim3(256), 0, 0, s, d, n); });
    run("blocked x4, 256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_blk<4>, dim3(n / 1024), dim3(256), 0, 0, s, d, n); });
    run("blocked x8, 256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_blk<8>, dim3(n / 2048), dim3(256), 0, 0, s, d, n); });
    run("blocked x16, 256", [&](float4 *s, float4 *d) { hipLaunchKernelGGL(k_blk<16>, dim3(n / 4096), dim3(256), 0, 0, s, d, n); });
    run("hipMemcpyDtoD", [&](float4 *s, float4 *d) { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
