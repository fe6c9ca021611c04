// gs_libm.hpp -- host/device restatement of the C library expf the reference's loader calls
// (std::exp on float, src/Splats.cpp:318-326), so the GPU load path (gs_scene_load_ply)
// reproduces the host loader bit for bit.
//
// The reference's std::exp(float) is glibc's expf (sysdeps/ieee754/flt-32/e_expf.c, glibc
// 2.27+; the container's glibc is 2.35): x*N/ln2 = k + r with N = 32, 2^(k/N) from a
// 32-entry table, 2^(r/N) from a cubic, all in double.  On x86-64 with FMA, glibc runs its
// FMA build, where the compiler fuses the reduction r = InvLn2N*x - kd (and the polynomial)
// into fmas; that is the sequence below.  Checked against the host's expf on every one of the
// 2^32 float inputs (0 mismatches; without the fused reduction: 2), see
// tests/test_libm_expf.py.  Table: tab[i] = bits(2^(i/32)) - (i << 47), the correctly rounded
// powers (generated with 60-digit decimal arithmetic).
#pragma once

#include <cstdint>
#include <cstring>

#ifndef __HIP__
#define GS_HD inline
#else
#define GS_HD __host__ __device__ inline
#endif

namespace gs {

GS_HD double libm_u2d(uint64_t u) {
    double d;
    std::memcpy(&d, &u, 8);
    return d;
}
GS_HD uint64_t libm_d2u(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}
GS_HD uint32_t libm_f2u(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

GS_HD float glibc_expf(float x) {
    constexpr uint64_t kTab[32] = {
        0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL,
        0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL,
        0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL,
        0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL,
        0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL,
        0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL,
        0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL,
        0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL};
    constexpr double N = 32.0;
    constexpr double InvLn2N = 0x1.71547652b82fep+0 * N;
    constexpr double C0 = 0x1.c6af84b912394p-5 / N / N / N, C1 = 0x1.ebfce50fac4f3p-3 / N / N,
                     C2 = 0x1.62e42ff0c52d6p-1 / N;
    constexpr double kShift = 0x1.8p+52;
    const uint32_t abstop = (libm_f2u(x) >> 20) & 0x7ff;
    if (abstop >= (libm_f2u(88.0f) >> 20)) {  // |x| >= 88 or NaN
        if (libm_f2u(x) == 0xff800000u) return 0.0f;            // -inf
        if (abstop >= (0x7f800000u >> 20)) return x + x;        // +inf, NaN
        if (x > 0x1.62e42ep6f) return __builtin_inff();         // overflow
        if (x < -0x1.9fe368p6f) return 0.0f;                    // underflow
    }
    const double xd = (double)x;
    double kd = __builtin_fma(InvLn2N, xd, kShift);
    const uint64_t ki = libm_d2u(kd);
    kd -= kShift;
    const double r = __builtin_fma(InvLn2N, xd, -kd);
    const double s = libm_u2d(kTab[ki % 32] + (ki << (52 - 5)));
    const double z = __builtin_fma(C0, r, C1);
    const double r2 = r * r;
    double y = __builtin_fma(C2, r, 1.0);
    y = __builtin_fma(z, r2, y);
    return (float)(y * s);
}

}  // namespace gs
