// Which SIMD does each wave of a 512-thread (8-wave) workgroup run on?  s_getreg HW_ID
// (gfx9: WAVE_ID [3:0], SIMD_ID [5:4], CU_ID [11:8]) for a few workgroups.
// Build: hipcc -O3 --offload-arch=gfx950 wave_simd.hip -o wave_simd
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void __launch_bounds__(512) k(int* out) {
    if ((threadIdx.x & 63) == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));   // HW_REG_HW_ID, all bits
        out[blockIdx.x * 8 + (threadIdx.x >> 6)] = (int)hw;
    }
}

int main() {
    int* d; hipMalloc(&d, 256 * 8 * 4);
    k<<<256, 512>>>(d);
    int h[256 * 8];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int hist[2][4] = {{0}};   // [pattern][...]
    for (int b = 0; b < 6; ++b) {
        printf("block %d:", b);
        for (int w = 0; w < 8; ++w) printf(" w%d->simd%d", w, (h[b * 8 + w] >> 4) & 3);
        printf("\n");
    }
    int same_w4 = 0, same_pair = 0;
    for (int b = 0; b < 256; ++b) {
        for (int w = 0; w < 4; ++w) same_w4 += ((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + w + 4] >> 4) & 3);
        for (int w = 0; w < 8; w += 2) same_pair += ((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + w + 1] >> 4) & 3);
    }
    printf("waves w and w+4 on one SIMD: %d / 1024;  waves 2i and 2i+1 on one SIMD: %d / 1024\n", same_w4, same_pair);
    (void)hist;
    return 0;
}
