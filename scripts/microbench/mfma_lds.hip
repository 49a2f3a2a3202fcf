// Microbenchmark: do LDS fragment reads (ds_read_b128) and 16x16x32 MFMAs overlap on a
// SIMD?  256 workgroups x 8 waves; per iteration every wave reads R fragments and issues
// M MFMAs on 20 accumulators.  MODE 0: reads + MFMAs; 1: MFMAs only; 2: reads only;
// 3: reads + MFMAs with the accumulators in AGPRs (inline asm, "+a").
// Build: hipcc -O3 --offload-arch=gfx950 mfma_lds.hip -o mfma_lds
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(512) k(float* out, int iters) {
    __shared__ __attribute__((aligned(16))) char lds[65536];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 65536 / 16; i += 512) reinterpret_cast<f16x8*>(lds)[i] = (f16x8){1, 1, 1, 1, 1, 1, 1, 1};
    __syncthreads();
    f32x4 acc[20];
    for (int i = 0; i < 20; ++i) acc[i] = (f32x4){0, 0, 0, 0};
    f16x8 fa[4], fb[5];
    // XOR-swizzled 128-B rows (chunk c of row r at slot c ^ ((r >> 1) & 7)): conflict-free b128 reads
    const int base = (lane & 15) * 128 + ((((lane >> 4)) ^ (((lane & 15) >> 1) & 7)) << 4) + wave * 8192;
    for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const f16x8*>(lds + base + i * 2048);
    for (int i = 0; i < 5; ++i) fb[i] = *reinterpret_cast<const f16x8*>(lds + (base ^ 4096) + i * 1024);
    for (int it = 0; it < iters; ++it) {
        if (MODE != 1) {
            const int o = (it & 1) * 8192;
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const f16x8*>(lds + ((base + i * 2048 + o) & 65535));
#pragma unroll
            for (int i = 0; i < 5; ++i) fb[i] = *reinterpret_cast<const f16x8*>(lds + ((base + 512 + i * 1024 + o) & 65535));
        }
        if (MODE == 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" :: "v"(fa[i]));
#pragma unroll
            for (int i = 0; i < 5; ++i) asm volatile("" :: "v"(fb[i]));
        } else if (MODE == 3) {
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int a = 0; a < 5; ++a)
                    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[a * 4 + b]) : "v"(fb[a]), "v"(fa[b]));
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int a = 0; a < 5; ++a)
                    acc[a * 4 + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[a], fa[b], acc[a * 4 + b], 0, 0, 0);
        }
    }
    float s = 0;
    for (int i = 0; i < 20; ++i) s += acc[i][0] + acc[i][3];
    if (s == 123.f) out[threadIdx.x] = s;
}

template <int MODE>
float run(float* out, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<MODE><<<256, 512>>>(out, iters);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k<MODE><<<256, 512>>>(out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 5 * 1e3;
}

int main() {
    float* out; hipMalloc(&out, 4096);
    const int iters = 2000;
    // per iteration per SIMD: 2 waves x 20 MFMA x 16 cycles = 640 cycles
    float t0 = run<0>(out, iters), t1 = run<1>(out, iters), t2 = run<2>(out, iters), t3 = run<3>(out, iters);
    printf("reads+mfma %.1f us | mfma only %.1f us | reads only %.1f us | reads+mfma(AGPR acc) %.1f us\n", t0, t1, t2, t3);
    printf("ideal mfma at 2.0 GHz: %.1f us\n", iters * 640 / 2.0e3);
    return 0;
}
