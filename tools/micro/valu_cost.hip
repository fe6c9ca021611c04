// Issue cost of the vector instructions k_draw's survivor step is made of (tools only):
// 6 waves per SIMD on every CU, each running 16 independent chains of one instruction type.
// Prints ns per wave-instruction per SIMD and that in cycles of the v_fma_f32 rate (2 cycles).
// ds_bpermute (a broadcast through the LDS crossbar) is LDS-throughput bound: ~8.5 v_fma's worth
// per wave-instruction per SIMD with every SIMD issuing them.
//   hipcc -O3 --offload-arch=gfx950 -o valu_cost valu_cost.hip && ./valu_cost
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 2048;
typedef float f2 __attribute__((ext_vector_type(2)));

template <int OP>
__global__ __launch_bounds__(64) void k(float *out, float a, float b, unsigned long long m) {
    float acc[16];
    f2 pacc[16];
    unsigned u[16];
    for (int i = 0; i < 16; ++i) {
        acc[i] = threadIdx.x * 0.001f + i;
        pacc[i] = f2{acc[i], acc[i] + 1.0f};
        u[i] = threadIdx.x + i;
    }
    const f2 pa = {a, a}, pb = {b, b};
    unsigned sacc = 0;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
            if (OP == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(pacc[i]) : "v"(pa), "v"(pb));
            if (OP == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(pacc[i]) : "v"(pa));
            if (OP == 3) {
                unsigned s;
                asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(s) : "v"(acc[i]));
                sacc ^= s;
            }
            if (OP == 4) asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(u[i]) : "s"((unsigned)m));
            if (OP == 5) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[i]) : "v"(i), "s"(m));
            if (OP == 6) asm volatile("v_exp_f32 %0, %0" : "+v"(acc[i]));
            if (OP == 7) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
            if (OP == 8) {
                unsigned long long s;
                asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(s) : "v"(acc[i]), "v"(a));
                sacc ^= (unsigned)s;
            }
            if (OP == 9) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
            if (OP == 10) {  // ds_bpermute broadcast of lane 5 (LDS crossbar, no LDS storage)
                unsigned r;
                asm volatile("ds_bpermute_b32 %0, %1, %2\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(20u), "v"(u[i]));
                u[i] ^= r;
            }
        }
    }
    float r = sacc;
    for (int i = 0; i < 16; ++i) r += acc[i] + pacc[i].x + pacc[i].y + (float)u[i];
    if (r == 1234.5f) out[threadIdx.x] = r;
}

template <int OP>
float run(float *out, int waves_per_simd) {
    const int grid = 256 * 4 * waves_per_simd;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k<OP>, dim3(grid), dim3(64), 0, 0, out, 1.0001f, 0.5f, 0x5555aaaa5555aaaaull);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    // ns per wave-instruction per SIMD
    return best * 1e6f / ((float)waves_per_simd * kIters * 16);
}

int main() {
    float *out;
    (void)hipMalloc(&out, 4096);
    const char *names[] = {"v_fma_f32", "v_pk_fma_f32", "v_pk_mul_f32", "v_readlane_b32", "v_mbcnt_lo", "v_cndmask(s)",
                           "v_exp_f32", "v_med3_f32", "v_cmp->sgpr", "v_add_f32", "ds_bpermute"};
    for (int w : {1, 2, 6}) {
        float ns[11] = {run<0>(out, w), run<1>(out, w), run<2>(out, w), run<3>(out, w), run<4>(out, w),
                        run<5>(out, w), run<6>(out, w), run<7>(out, w), run<8>(out, w), run<9>(out, w),
                        run<10>(out, w)};
        std::printf("waves/SIMD %d\n", w);
        for (int i = 0; i < 11; ++i)
            std::printf("  %-16s %.3f ns  = %.2f x v_fma (%.2f cyc at the fma's 2)\n", names[i], ns[i], ns[i] / ns[0],
                        2.0f * ns[i] / ns[0]);
    }
    return 0;
}
