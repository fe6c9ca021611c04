// Random-gather throughput microbenchmark (diagnostics only, not part of the product).
// gather: out[i] = table[idx[i]] for float4 / float2 / float tables of several sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

template <typename T>
__global__ void k_gather(const T* __restrict__ table, const unsigned* __restrict__ idx, float* __restrict__ out, int n) {
    int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    T v = table[idx[i]];
    const float* f = reinterpret_cast<const float*>(&v);
    float s = 0.f;
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) s += f[k];
    out[i] = s;
}

template <typename T>
void run(size_t table_bytes, int n, unsigned* d_idx, float* d_out, std::vector<unsigned>& h_idx) {
    size_t cnt = table_bytes / sizeof(T);
    T* d_t;
    hipMalloc(&d_t, cnt * sizeof(T));
    hipMemset(d_t, 0, cnt * sizeof(T));
    std::mt19937 rng(1);
    for (int i = 0; i < n; ++i) h_idx[i] = rng() % cnt;
    hipMemcpy(d_idx, h_idx.data(), n * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_gather<T>, dim3((n + 255) / 256), dim3(256), 0, 0, d_t, d_idx, d_out, n);
    hipEventRecord(a);
    const int R = 10;
    for (int w = 0; w < R; ++w) hipLaunchKernelGGL(k_gather<T>, dim3((n + 255) / 256), dim3(256), 0, 0, d_t, d_idx, d_out, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= R;
    printf("elem %2zuB table %7.1f MB: %8.1f us  %7.1f Ggathers/s\n", sizeof(T), table_bytes / 1e6, ms * 1e3,
           n / (ms * 1e-3) / 1e9);
    hipFree(d_t);
}

int main() {
    const int n = 10'000'000;
    unsigned* d_idx;
    float* d_out;
    hipMalloc(&d_idx, n * 4);
    hipMalloc(&d_out, n * 4);
    std::vector<unsigned> h(n);
    for (size_t mb : {2, 16, 64, 128, 256, 512, 1024}) {
        run<float4>(mb << 20, n, d_idx, d_out, h);
        run<float2>(mb << 20, n, d_idx, d_out, h);
        run<float>(mb << 20, n, d_idx, d_out, h);
    }
    return 0;
}
