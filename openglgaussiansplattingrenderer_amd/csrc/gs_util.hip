// gs_util.hip -- measurement helpers of the C ABI (not on the frame path).
//
// gs_stream_copy_gbs: the HBM stream-copy rate of this GPU, measured in the same process as the
// kernels it is compared with (bench.py's roofline.frac_of_copy): a float4 copy (one per lane,
// non-temporal) between two buffers far beyond the 256 MiB Infinity Cache, bytes read + written per second.
// MI355X_MICROARCH.md quotes 6.29 TB/s for a float4 copy against the 8.0 TB/s spec.
#include "gs_internal.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

namespace {

// one float4 per lane, non-temporal loads and stores (tools/micro/copy_bw.hip on MI355X, 1 GiB:
// 6.58 TB/s; temporal 6.23; grid-stride loops of 4-8 float4 per lane 4.4-4.7; hipMemcpy 4.7)
typedef float f4v __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_copy(const f4v *__restrict__ src, f4v *__restrict__ dst, size_t n4) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

}  // namespace

extern "C" int gs_stream_copy_gbs(gs_ctx *ctx, size_t bytes, int reps, double *gbs_median, double *gbs_best) {
    if (!ctx) return gs::set_error(nullptr, GS_ERR_INVALID, "ctx is null");
    if (!gbs_median || reps < 1 || bytes < 4096) return gs::set_error(ctx, GS_ERR_INVALID, "gs_stream_copy_gbs: bad argument");
    if (int rc = gs::ctx_use_device(ctx)) return rc;  // the buffers on the ctx's GPU
    if (int rc = gs_sync(ctx)) return rc;  // nothing of the ctx's frames shares the GPU with it
    const size_t n4 = bytes / 16;
    f4v *a = nullptr, *b = nullptr;
    hipStream_t s = (hipStream_t)gs_stream(ctx);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto done = [&](int rc) {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (a) (void)hipFree(a);
        if (b) (void)hipFree(b);
        return rc;
    };
    if (hipMalloc(&a, n4 * 16) != hipSuccess || hipMalloc(&b, n4 * 16) != hipSuccess)
        return done(gs::set_error(ctx, GS_ERR_NOMEM, "gs_stream_copy_gbs: out of device memory"));
    if (hipMemsetAsync(a, 0, n4 * 16, s) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess)
        return done(gs::set_error(ctx, GS_ERR_HIP, "gs_stream_copy_gbs: setup failed"));
    const dim3 grid((unsigned)((n4 + 255) / 256));
    std::vector<double> r;
    for (int i = 0; i < reps + 2; ++i) {
        const bool ab = (i & 1) == 0;  // alternate directions: neither buffer stays cached
        (void)hipEventRecord(e0, s);
        hipLaunchKernelGGL(k_stream_copy, grid, dim3(256), 0, s, ab ? a : b, ab ? b : a, n4);
        (void)hipEventRecord(e1, s);
        if (hipEventSynchronize(e1) != hipSuccess)
            return done(gs::set_error(ctx, GS_ERR_HIP, "gs_stream_copy_gbs: copy failed"));
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (i >= 2 && ms > 0.f) r.push_back(2.0 * (double)(n4 * 16) / (ms * 1e-3) / 1e9);
    }
    if (r.empty()) return done(gs::set_error(ctx, GS_ERR_HIP, "gs_stream_copy_gbs: no timing"));
    std::sort(r.begin(), r.end());
    *gbs_median = r[r.size() / 2];
    if (gbs_best) *gbs_best = r.back();
    return done(GS_OK);
}
