// Throughput of per-block histogram reduction on MI355X: B blocks each add 1280 counters
// (LDS-aggregated) into one global histogram with device-scope atomics, vs writing partial
// rows.  hipcc --offload-arch=gfx950 -O3 atomics_bench.hip -o atomics_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_atomic(uint32_t *h, int bins) {
    for (int i = threadIdx.x; i < bins; i += blockDim.x) atomicAdd(&h[i], (uint32_t)(blockIdx.x + i) & 7u);
}
__global__ void k_rows(uint32_t *rows, int bins) {
    for (int i = threadIdx.x; i < bins; i += blockDim.x) rows[(size_t)blockIdx.x * bins + i] = (blockIdx.x + i) & 7u;
}
__global__ void k_reduce1(const uint32_t *rows, uint32_t *h, int nb, int bins) {
    for (int i = threadIdx.x; i < bins; i += blockDim.x) {
        uint32_t s = 0;
        for (int b = 0; b < nb; ++b) s += rows[(size_t)b * bins + i];
        h[i] = s;
    }
}
int main() {
    uint32_t *h, *rows;
    hipMalloc(&h, 1 << 20);
    hipMalloc(&rows, 64 << 20);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int bins : {1024, 1280}) {
        for (int nb : {256, 512, 614, 2456}) {
            float best = 1e9, best2 = 1e9, best3 = 1e9;
            for (int rep = 0; rep < 20; ++rep) {
                hipMemset(h, 0, bins * 4);
                hipEventRecord(a);
                hipLaunchKernelGGL(k_atomic, dim3(nb), dim3(256), 0, 0, h, bins);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                best = ms < best ? ms : best;
                hipEventRecord(a);
                hipLaunchKernelGGL(k_rows, dim3(nb), dim3(256), 0, 0, rows, bins);
                hipEventRecord(b);
                hipEventSynchronize(b);
                hipEventElapsedTime(&ms, a, b);
                best2 = ms < best2 ? ms : best2;
                hipEventRecord(a);
                hipLaunchKernelGGL(k_reduce1, dim3(1), dim3(1024), 0, 0, rows, h, nb, bins);
                hipEventRecord(b);
                hipEventSynchronize(b);
                hipEventElapsedTime(&ms, a, b);
                best3 = ms < best3 ? ms : best3;
            }
            printf("bins %d blocks %d: global atomics %.1f us (%.0f Matomic/s); partial rows %.1f us + 1-block reduce %.1f us\n",
                   bins, nb, best * 1e3, bins * (double)nb / (best * 1e3), best2 * 1e3, best3 * 1e3);
        }
    }
    return 0;
}
