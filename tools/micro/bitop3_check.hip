// Checks the v_bitop3 truth-table convention on the GPU (tools only): for acc | (s ^ b), which
// immediate gives the C expression's result with operands (acc, s, sgpr b)?
#include <hip/hip_runtime.h>
#include <cstdio>
template <int T>
__device__ unsigned bop(unsigned a, unsigned s, unsigned b) {
    unsigned r;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:%4" : "=v"(r) : "v"(a), "v"(s), "s"(b), "i"(T));
    return r;
}
__global__ void k(unsigned *out, unsigned b) {
    const unsigned t = threadIdx.x;
    const unsigned a = t * 2654435761u, s = (t & 1) ? 0xffffffffu : 0u;
    const unsigned ref = a | (s ^ b);
    out[4 * t + 0] = ref;
    out[4 * t + 1] = bop<0xf6>(a, s, b);
    out[4 * t + 2] = bop<0xde>(a, s, b);
    out[4 * t + 3] = bop<0xbe>(a, s, b);
}
int main() {
    unsigned *d, h[256 * 4];
    (void)hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 0, 0, d, 0x5a5a1234u);
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int ok[3] = {1, 1, 1};
    for (int t = 0; t < 256; ++t)
        for (int j = 0; j < 3; ++j) ok[j] &= h[4 * t + 1 + j] == h[4 * t];
    std::printf("0xf6 %d  0xde %d  0xbe %d\n", ok[0], ok[1], ok[2]);
    return 0;
}
