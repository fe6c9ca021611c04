// Reference point for the sort's beyond-cache rate (not product code): rocPRIM's radix_sort_pairs
// (onesweep) on N uniform 32-bit keys with 32-bit values, hipEvents, median of 10.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/rocprim_sort.hip -o tools/micro/rocprim_sort
//   tools/micro/rocprim_sort [N]
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (size_t)1 << 26;
    std::vector<uint32_t> hk(n), hv(n);
    uint32_t x = 12345u;
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13, x ^= x >> 17, x ^= x << 5;
        hk[i] = x;
        hv[i] = (uint32_t)i;
    }
    uint32_t *k0, *v0, *k1, *v1;
    if (hipMalloc(&k0, n * 4) || hipMalloc(&v0, n * 4) || hipMalloc(&k1, n * 4) || hipMalloc(&v1, n * 4)) return 1;
    size_t tmp_bytes = 0;
    if (rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, v0, v1, n)) return 2;
    void *tmp;
    if (hipMalloc(&tmp, tmp_bytes)) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    std::vector<float> ms;
    for (int r = 0; r < 12; ++r) {
        (void)hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice);
        (void)hipEventRecord(a, 0);
        if (rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n)) return 3;
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, a, b);
        if (r >= 2) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::vector<uint32_t> out(n);
    (void)hipMemcpy(out.data(), k1, n * 4, hipMemcpyDeviceToHost);
    const bool ok = std::is_sorted(out.begin(), out.end());
    const double med = ms[ms.size() / 2];
    printf("{\"n\": %zu, \"ms_pairs\": %.4f, \"gkeys_per_s\": %.2f, \"hbm_frac_algorithmic_68B\": %.4f, \"sorted_ok\": %s, "
           "\"temp_bytes\": %zu}\n",
           n, med, n / (med * 1e-3) / 1e9, 68.0 * n / (med * 1e-3) / 8e12, ok ? "true" : "false", tmp_bytes);
    return ok ? 0 : 4;
}
