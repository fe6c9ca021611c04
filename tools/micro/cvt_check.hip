// Checks that v_cvt_i32_f32 is GLSL int(float) as the oracle states it (tools only): NaN -> 0,
// saturation at INT_MIN / INT_MAX, truncation toward zero -- against the explicit branchy form,
// over special values and 2^26 sampled bit patterns (every exponent, both signs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ int f2i_ref(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return (-2147483647 - 1);
    return (int)f;
}
__device__ int f2i_cvt(float f) {
    int r;
    asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(f));
    return r;
}
__global__ void k(unsigned long long *bad, uint32_t base) {
    const uint32_t i = base + blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t bits = i * 64u + (i % 64u);  // 1 pattern in 64, all residues
    const float f = __uint_as_float(bits);
    if (f2i_ref(f) != f2i_cvt(f)) atomicAdd(bad, 1ull);
}
__global__ void special(int *out) {
    const float v[10] = {__int_as_float(0x7fc00000), __int_as_float(0xffc00001), __int_as_float(0x7f800000),
                         __int_as_float(0xff800000), 2147483648.0f, -2147483904.0f, -2147483648.0f, 2.5f, -2.5f, -0.0f};
    const int t = threadIdx.x;
    if (t < 10) {
        out[2 * t] = f2i_ref(v[t]);
        out[2 * t + 1] = f2i_cvt(v[t]);
    }
}
int main() {
    unsigned long long *d, h = 0;
    int *o, ho[20];
    (void)hipMalloc(&d, 8);
    (void)hipMalloc(&o, sizeof ho);
    (void)hipMemset(d, 0, 8);
    for (uint32_t b = 0; b < (1u << 26); b += (1u << 24))
        hipLaunchKernelGGL(k, dim3((1u << 24) / 256), dim3(256), 0, 0, d, b);
    hipLaunchKernelGGL(special, dim3(1), dim3(64), 0, 0, o);
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
    int sp = 0;
    for (int t = 0; t < 10; ++t) sp += ho[2 * t] != ho[2 * t + 1];
    std::printf("cvt_check: %llu mismatches over 2^26 patterns, %d of 10 special values differ\n", h, sp);
    for (int t = 0; t < 10; ++t) std::printf("  ref %d cvt %d\n", ho[2 * t], ho[2 * t + 1]);
    return h || sp;
}
