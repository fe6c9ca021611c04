// gs_load.hip -- GPU load path: the reference's per-splat activations
// (Splats::loadSplats, src/Splats.cpp:289-331) and covariance (computeCovarianceMatrices /
// computeCovarianceMatrix, src/Splats.cpp:414-479) for raw ply records already in device
// memory.  Every float operation is the host loader's (gs_host.cpp activate_one /
// covariance3d) in the same order, exp is glibc's expf restated (gs_libm.hpp), division and
// sqrt are correctly rounded (HIP's default) and nothing is contracted (-ffp-contract=off),
// so the scene is bit-identical to gs_ply_load + gs_covariance3d + gs_scene_create.
#include "gs_internal.hpp"
#include "gs_libm.hpp"

#include <hip/hip_runtime.h>

namespace gs {

namespace {

__global__ __launch_bounds__(256) void k_ply_activate(const float *__restrict__ rec, int count, int base, int n,
                                                      float *__restrict__ soa, float4 *__restrict__ colour) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= count) return;
    const float *r = rec + (size_t)j * kPlyFloats;
    const size_t i = (size_t)base + j, nn = (size_t)n;
    // :289-300 means (normals r[3..5] and f_rest r[9..53] are read and dropped)
    soa[i] = r[0];
    soa[nn + i] = r[1];
    soa[2 * nn + i] = r[2];
    // :304-312 colour = (0.5 + SH_C0 * f_dc) * 255, alpha 1
    const float SH_C0 = 0.28209479177387814f;
    colour[i] = make_float4((0.5f + (SH_C0 * r[6])) * 255.f, (0.5f + (SH_C0 * r[7])) * 255.f,
                            (0.5f + (SH_C0 * r[8])) * 255.f, 1.f);
    // :314-316 opacity = sigmoid(logit)
    const float opac = (1 / (1 + glibc_expf(-r[54])));
    // :318-326 scale = exp(log scale); :328-331 rotation normalised
    const float sx = glibc_expf(r[55]), sy = glibc_expf(r[56]), sz = glibc_expf(r[57]);
    const float q0 = r[58], q1 = r[59], q2 = r[60], q3 = r[61];
    const float length = sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
    const float rr = q0 / length, x = q1 / length, y = q2 / length, z = q3 / length;
    // :440-479 T = S * R (glm mat3, column-major), Sigma = transpose(T) * T
    const float S[3][3] = {{sx, 0, 0}, {0, sy, 0}, {0, 0, sz}};
    const float R[3][3] = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - rr * z), 2.f * (x * z + rr * y)},
                           {2.f * (x * y + rr * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - rr * x)},
                           {2.f * (x * z - rr * y), 2.f * (y * z + rr * x), 1.f - 2.f * (x * x + y * y)}};
    float M[3][3], Sig[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < 3; ++q) M[c][q] = S[0][q] * R[c][0] + S[1][q] * R[c][1] + S[2][q] * R[c][2];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int q = 0; q < 3; ++q) Sig[c][q] = M[q][0] * M[c][0] + M[q][1] * M[c][1] + M[q][2] * M[c][2];
    // the shape record (SceneDev): covariance upper triangle and opacity
    float *shape = soa + scene_shape_offset(nn) + (size_t)kShapeFloats * i;
    const float rs[kShapeFloats] = {Sig[0][0], Sig[0][1], Sig[0][2], Sig[1][1], Sig[1][2], Sig[2][2], opac};
#pragma unroll
    for (int c = 0; c < kShapeFloats; ++c) shape[c] = rs[c];
}

}  // namespace

void launch_ply_activate(hipStream_t s, const float *rec, int count, int base, int n, float *soa, float4 *colour) {
    if (count > 0)
        hipLaunchKernelGGL(k_ply_activate, dim3((count + 255) / 256), dim3(256), 0, s, rec, count, base, n, soa, colour);
}

}  // namespace gs
