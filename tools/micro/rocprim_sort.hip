// rocprim_sort.hip -- same-box bar for the radix sort (tools only, never linked into the product):
// rocprim::radix_sort_pairs (header-only rocPRIM of the image) against libgsplat_hip's
// gs_sort_pairs_u32 on the same (u32 key, u32 value) inputs, hipEvent-timed, median of R.
//   build: tools/micro/build_rocprim_sort.sh     run: tools/micro/rocprim_sort [R]
// Inputs: the reference's sortTests keys (src/utils.cpp:49-63 with srand(20), n = 5,119,993,
// tests/sortTests.cpp:181), render-like 10M (tile + depth floats), uniform 32-bit 10M and 64M
// (64M pairs = 512 MB with the alternate buffers: beyond the 256 MiB Infinity Cache).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/gsplat.h"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

static std::vector<uint32_t> sorttests_keys(int n) {
    std::vector<uint32_t> k(n);
    srand(20);  // src/utils.cpp:49-63
    for (int i = 0; i < n; i++) {
        int random = rand() % 255;
        float f = (float)rand() / RAND_MAX + random + 0.5f;
        std::memcpy(&k[i], &f, 4);
    }
    return k;
}

static std::vector<uint32_t> render_like(int n, uint64_t seed) {
    std::mt19937_64 g(seed);
    std::vector<uint32_t> k(n);
    for (int i = 0; i < n; ++i) {
        float f = (float)(g() % 256) + 0.96f + 0.03f * (float)((g() >> 11) * (1.0 / 9007199254740992.0));
        std::memcpy(&k[i], &f, 4);
    }
    return k;
}

static std::vector<uint32_t> uniform32(int n, uint64_t seed) {
    std::mt19937_64 g(seed);
    std::vector<uint32_t> k(n);
    for (auto &x : k) x = (uint32_t)(g() >> 32);
    return k;
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? std::atoi(argv[1]) : 20;
    const int only = argc > 2 ? std::atoi(argv[2]) : -1;  // run one case (PMC passes)
    struct Case {
        const char *name;
        std::vector<uint32_t> keys;
    };
    std::vector<Case> cases;
    cases.push_back({"sortTests 5.12M", sorttests_keys(32 * 16 * 10000 - 7)});
    cases.push_back({"render-like 10M", render_like(10000000, 1)});
    cases.push_back({"uniform32 10M", uniform32(10000000, 2)});
    cases.push_back({"uniform32 64M", uniform32(64 << 20, 3)});
    gs_ctx *ctx = nullptr;
    if (gs_ctx_create(0, &ctx)) {
        std::fprintf(stderr, "gs_ctx_create: %s\n", gs_last_error(nullptr));
        return 1;
    }
    hipStream_t s = (hipStream_t)gs_stream(ctx);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (size_t ci = 0; ci < cases.size(); ++ci) {
        if (only >= 0 && (int)ci != only) continue;
        auto &c = cases[ci];
        const size_t n = c.keys.size();
        std::vector<uint32_t> iota(n);
        for (size_t i = 0; i < n; ++i) iota[i] = (uint32_t)i;
        // expected: stable argsort by key
        std::vector<uint32_t> exp(iota);
        std::stable_sort(exp.begin(), exp.end(), [&](uint32_t a, uint32_t b) { return c.keys[a] < c.keys[b]; });
        uint32_t *k0, *v0, *k1, *v1, *kw, *vw;
        CK(hipMalloc(&k0, n * 4));
        CK(hipMalloc(&v0, n * 4));
        CK(hipMalloc(&k1, n * 4));
        CK(hipMalloc(&v1, n * 4));
        CK(hipMalloc(&kw, n * 4));
        CK(hipMalloc(&vw, n * 4));
        CK(hipMemcpy(k0, c.keys.data(), n * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(v0, iota.data(), n * 4, hipMemcpyHostToDevice));
        size_t tb = 0;
        CK(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, n, 0, 32, s));
        void *tmp;
        CK(hipMalloc(&tmp, tb));
        std::vector<float> tr, tg;
        for (int r = 0; r < R + 3; ++r) {
            CK(hipEventRecord(e0, s));
            CK(rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, n, 0, 32, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) tr.push_back(ms);
        }
        std::vector<uint32_t> got(n);
        CK(hipMemcpy(got.data(), v1, n * 4, hipMemcpyDeviceToHost));
        const bool ok_r = got == exp;
        for (int r = 0; r < R + 3; ++r) {  // gs_sort_pairs_u32 sorts in place: fresh copies each time
            CK(hipMemcpyAsync(kw, k0, n * 4, hipMemcpyDeviceToDevice, s));
            CK(hipMemcpyAsync(vw, v0, n * 4, hipMemcpyDeviceToDevice, s));
            if (gs_sort_pairs_u32(ctx, kw, vw, (int64_t)n)) {
                std::fprintf(stderr, "gs_sort_pairs_u32: %s\n", gs_last_error(ctx));
                return 1;
            }
            float ms;
            if (gs_last_kernel_ms(ctx, GS_KERNEL_SORT, &ms)) return 1;
            if (r >= 3) tg.push_back(ms);
        }
        CK(hipMemcpy(got.data(), vw, n * 4, hipMemcpyDeviceToHost));
        const bool ok_g = got == exp;
        std::sort(tr.begin(), tr.end());
        std::sort(tg.begin(), tg.end());
        const double mr = tr[tr.size() / 2], mg = tg[tg.size() / 2];
        std::printf("%-18s n=%10zu  rocprim %8.1f us (%6.2f Gkeys/s) ok=%d   gsplat %8.1f us (%6.2f Gkeys/s) ok=%d   "
                    "gsplat/rocprim %.2f\n",
                    c.name, n, mr * 1e3, n / mr / 1e6, ok_r, mg * 1e3, n / mg / 1e6, ok_g, mg / mr);
        std::fflush(stdout);
        for (void *p : {(void *)k0, (void *)v0, (void *)k1, (void *)v1, (void *)kw, (void *)vw, tmp}) CK(hipFree(p));
    }
    gs_ctx_destroy(ctx);
    return 0;
}
