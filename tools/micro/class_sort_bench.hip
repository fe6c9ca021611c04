// Probe (not product code): gs_sort.hip's k_class_sort alone on synthetic buckets -- 256 buckets of
// M keys each (bucket b: bits of b + U[0,1)), placement deltas 0 -- hipEvents, median of 20; checks
// that every bucket comes out stably sorted.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include tools/micro/class_sort_bench.hip -o /tmp/csb
//   /tmp/csb M [M ...]
#include "../../openglgaussiansplattingrenderer_amd/csrc/gs_sort.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char **argv) {
    for (int a = 1; a < argc; ++a) {
        const uint32_t M = (uint32_t)atoi(argv[a]);
        const size_t n = (size_t)256 * M;
        std::vector<uint32_t> hk(n), hv(n), rt(256, M);
        uint32_t x = 12345u + M;
        for (size_t i = 0; i < n; ++i) {
            x ^= x << 13, x ^= x >> 17, x ^= x << 5;
            const float f = (float)(i / M) + (float)(x >> 8) * (1.0f / 16777216.0f);
            std::memcpy(&hk[i], &f, 4);
            hv[i] = (uint32_t)i;
        }
        uint32_t *k0, *v0, *k1, *v1, *vo, *rtd;
        int32_t *delta;
        if (hipMalloc(&k0, n * 4) || hipMalloc(&v0, n * 4) || hipMalloc(&k1, n * 4) || hipMalloc(&v1, n * 4) ||
            hipMalloc(&vo, n * 4) || hipMalloc(&rtd, 256 * 4) || hipMalloc(&delta, 257 * 4))
            return 1;
        (void)hipMemcpy(rtd, rt.data(), 256 * 4, hipMemcpyHostToDevice);
        (void)hipMemset(delta, 0, 257 * 4);
        gs::PrefixDev pd{};
        pd.delta = delta;
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        std::vector<float> ms;
        for (int it = 0; it < 23; ++it) {
            (void)hipMemcpy(k0, hk.data(), n * 4, hipMemcpyHostToDevice);
            (void)hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(gs::k_class_sort, dim3(256), dim3(gs::kCsWaves * 64), 0, 0, k0, v0, k1, v1, vo, rtd, pd);
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float t = 0.f;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (it >= 3) ms.push_back(t);
        }
        std::vector<uint32_t> out(n);
        (void)hipMemcpy(out.data(), vo, n * 4, hipMemcpyDeviceToHost);
        bool ok = true;
        for (size_t i = 0; i < n && ok; ++i) {
            if (out[i] >= n || out[i] / M != i / M) ok = false;
            else if (i % M && (hk[out[i]] < hk[out[i - 1]] || (hk[out[i]] == hk[out[i - 1]] && out[i] < out[i - 1]))) ok = false;
        }
        std::sort(ms.begin(), ms.end());
        printf("M %6u  keys %8zu  k_class_sort %.4f ms (min %.4f)  %s\n", M, n, ms[ms.size() / 2], ms[0], ok ? "sorted" : "WRONG");
        (void)hipFree(k0), (void)hipFree(v0), (void)hipFree(k1), (void)hipFree(v1), (void)hipFree(vo), (void)hipFree(rtd),
            (void)hipFree(delta);
    }
    return 0;
}
