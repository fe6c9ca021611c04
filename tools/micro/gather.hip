// Random-gather microbenchmark and FETCH_SIZE calibration (diagnostics only, not the product).
// gather: out[i] = sum of the floats of table[idx[i]] for 4 / 8 / 16 / 32-byte elements (the
// blend's access widths: 4-B sorted values, 8-B cull boxes, 12/16-B colours, 28/32-B records)
// from tables inside (64 MiB) and beyond (1 GiB) the 256 MiB Infinity Cache, n = 10M gathers.
// Each config launches `reps` times; stdout lists the configs in dispatch order, so a
// rocprofv3 --pmc run (tools/micro/gather_pmc.sh) maps each dispatch to its known byte counts:
//   idx stream 4n B (coalesced), out stream 4n B, n gathers of the element width.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

template <int B>
struct alignas(B < 16 ? B : 16) Elem {
    float f[B / 4];
};

template <int B>
__global__ __launch_bounds__(256) void k_gather(const Elem<B> *__restrict__ table, const unsigned *__restrict__ idx,
                                                float *__restrict__ out, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const Elem<B> v = table[idx[i]];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < B / 4; ++k) s += v.f[k];
    out[i] = s;
}

template <int B>
void run(size_t table_bytes, int n, unsigned *d_idx, float *d_out, std::vector<unsigned> &h_idx, int reps) {
    const size_t cnt = table_bytes / B;
    Elem<B> *d_t;
    if (hipMalloc(&d_t, cnt * B) != hipSuccess) std::exit(1);
    (void)hipMemset(d_t, 0, cnt * B);
    std::mt19937 rng(1);
    for (int i = 0; i < n; ++i) h_idx[i] = rng() % cnt;
    (void)hipMemcpy(d_idx, h_idx.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float best = 1e30f;
    for (int w = 0; w < reps; ++w) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(k_gather<B>, dim3((n + 255) / 256), dim3(256), 0, 0, d_t, d_idx, d_out, n);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (w > 0 && ms < best) best = ms;
    }
    std::printf("CONFIG elem=%d table_mb=%.1f n=%d reps=%d best_us=%.1f ggathers=%.2f\n", B, table_bytes / 1048576.0, n,
                reps, best * 1e3, n / (best * 1e-3) / 1e9);
    std::fflush(stdout);
    (void)hipFree(d_t);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

int main(int argc, char **argv) {
    const int n = 10'000'000, reps = argc > 1 ? std::atoi(argv[1]) : 3;
    unsigned *d_idx;
    float *d_out;
    if (hipMalloc(&d_idx, (size_t)n * 4) != hipSuccess || hipMalloc(&d_out, (size_t)n * 4) != hipSuccess) return 1;
    std::vector<unsigned> h(n);
    for (size_t mb : {64, 1024}) {
        run<4>(mb << 20, n, d_idx, d_out, h, reps);
        run<8>(mb << 20, n, d_idx, d_out, h, reps);
        run<16>(mb << 20, n, d_idx, d_out, h, reps);
        run<32>(mb << 20, n, d_idx, d_out, h, reps);
    }
    return 0;
}
