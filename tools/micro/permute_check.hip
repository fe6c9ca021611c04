// ds_permute_b32 (forward permute) semantics on gfx950: what a lane that no active lane writes to
// receives (0, or its old value?), with an exec-masked source set.  Not product code.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/permute_check.hip -o tools/micro/permute_check
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k(int *out) {
    const int lane = threadIdx.x;
    int r = 1000 + lane;  // the destination's prior value
    if (lane < 8) r = __builtin_amdgcn_ds_permute((lane * 2) << 2, 7 + lane);  // lanes 0-7 push to 0,2,...,14
    out[lane] = r;
    // full-exec permute where only lanes < 8 have a meaningful target: the others push to lane 63
    int r2 = __builtin_amdgcn_ds_permute(lane < 8 ? (lane * 2) << 2 : 63 << 2, lane < 8 ? 7 + lane : -1);
    out[64 + lane] = r2;
}

int main() {
    int *d;
    if (hipMalloc(&d, 128 * 4)) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    int h[128];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost)) return 2;
    printf("exec-masked (lanes 0-7 push to 2*lane; lanes >= 8 inactive):");
    for (int i = 0; i < 20; ++i) printf(" %d", h[i]);
    printf("\nfull exec (lanes >= 8 push -1 to lane 63):");
    for (int i = 0; i < 20; ++i) printf(" %d", h[64 + i]);
    printf(" ... lane63=%d\n", h[127]);
    return 0;
}
