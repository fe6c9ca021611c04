// Is the f32 division's Newton core, with the reciprocal of the denominator computed once, bit-for-
// bit the compiler's correctly rounded a / b wherever v_div_scale would not scale (|a|, |b| in
// [2^-40, 2^40])?  Random operands (log-uniform magnitudes, random signs), N per thread; counts
// mismatches.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/div_check.hip -o tools/micro/div_check
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ uint32_t xs(uint32_t &s) {
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return s;
}
__device__ __forceinline__ float rnd(uint32_t &s) {
    // sign, exponent in [-40, 39], random mantissa
    const uint32_t m = xs(s) & 0x7fffffu, e = (uint32_t)(127 - 40) + (xs(s) % 80u), sg = xs(s) & 0x80000000u;
    return __uint_as_float(sg | (e << 23) | m);
}
__global__ void k(unsigned long long *bad, int per, float *ex) {
    uint32_t s = 0x9e3779b9u ^ (blockIdx.x * 256u + threadIdx.x) * 2654435761u;
    unsigned long long nb = 0;
    for (int i = 0; i < per; ++i) {
        const float b = rnd(s);
        const float r0 = __builtin_amdgcn_rcpf(b), nbv = -b;
        const float r1 = __builtin_fmaf(__builtin_fmaf(nbv, r0, 1.0f), r0, r0);
        for (int j = 0; j < 4; ++j) {
            const float a = rnd(s);
            const float m = a * r1;
            const float f3 = __builtin_fmaf(__builtin_fmaf(nbv, m, a), r1, m);
            const float q = __builtin_fmaf(__builtin_fmaf(nbv, f3, a), r1, f3);
            const float ref = a / b;
            if (__float_as_uint(q) != __float_as_uint(ref)) {
                ++nb;
                ex[0] = a, ex[1] = b;
            }
        }
        // 1 / b as the compiler writes it
        const float one = 1.0f;
        const float m = one * r1;
        const float f3 = __builtin_fmaf(__builtin_fmaf(nbv, m, one), r1, m);
        const float q = __builtin_fmaf(__builtin_fmaf(nbv, f3, one), r1, f3);
        if (__float_as_uint(q) != __float_as_uint(1.0f / b)) ++nb;
    }
    atomicAdd(bad, nb);
}

int main() {
    unsigned long long *d, h = 0;
    float *ex, hx[2] = {0, 0};
    if (hipMalloc(&d, 8) || hipMalloc(&ex, 8) || hipMemset(d, 0, 8) || hipMemset(ex, 0, 8)) return 1;
    const int blocks = 4096, per = 4096;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, per, ex);
    if (hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost) || hipMemcpy(hx, ex, 8, hipMemcpyDeviceToHost)) return 2;
    const double n = (double)blocks * 256 * per * 5;
    printf("divisions checked %.3g, mismatches %llu (last a=%g b=%g)\n", n, h, hx[0], hx[1]);
    return h ? 3 : 0;
}
