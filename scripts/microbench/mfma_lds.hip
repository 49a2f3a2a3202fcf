// Microbenchmark: do LDS fragment reads (ds_read_b128) and 16x16x32 MFMAs overlap on a
// SIMD?  256 workgroups x 8 waves; per iteration every wave reads R fragments and issues
// M MFMAs on 20 accumulators.  MODE 0: reads + MFMAs; 1: MFMAs only; 2: reads only;
// 3: reads + MFMAs with the accumulators in AGPRs (inline asm, "+a"); 4: ping-pong -- two
// wave groups (waves 0-3 / 4-7, one of each per SIMD) one barrier apart, each phase a read
// section then an MFMA section closed by barriers; 5: as 4 without s_setprio.
// Build: hipcc -O3 --offload-arch=gfx950 mfma_lds.hip -o mfma_lds
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) void* lptr_t;

// MODE 6 + NP: ping-pong with NP LDS-DMA pieces (buffer_load_dwordx4 ... lds, 1 KiB per
// wave-instruction, 8 rows x 128 B of a 64 MB source at a 640-B row pitch, as the conv's
// A operand) issued in every read section, into a separate 32 KiB LDS area
template <int MODE, int NP = 0>
__global__ void __launch_bounds__(512) k(float* out, int iters, const char* src = nullptr) {
    __shared__ __attribute__((aligned(16))) char lds[65536 + 32768];
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
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), 0, 64 << 20, 0x00020000);
    const unsigned soff0 = (unsigned)(((blockIdx.x * 64 + wave * 8 + (lane >> 3)) * 640 + (lane & 7) * 16));
    if (MODE >= 4) {
        const int grp = wave >> 2;
        if (grp) __builtin_amdgcn_s_barrier();
        for (int it = 0; it < iters; ++it) {
            const int o = (it & 1) * 8192;
#pragma unroll
            for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const f16x8*>(lds + ((base + i * 2048 + o) & 65535));
#pragma unroll
            for (int i = 0; i < 5; ++i) fb[i] = *reinterpret_cast<const f16x8*>(lds + ((base + 512 + i * 1024 + o) & 65535));
#pragma unroll
            for (int pc = 0; pc < NP; ++pc) {
                const unsigned off = (soff0 + (unsigned)((it * NP + pc) % 512) * 65536u) & ((64u << 20) - 1);
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lptr_t)(lds + 65536 + ((wave * NP + pc) & 31) * 1024),
                                                         16, off, 0, 0, 0);
            }
            if (NP) __builtin_amdgcn_s_waitcnt((NP & 15) | (7 << 4) | (15 << 8) | ((NP >> 4) << 14));   // vmcnt(NP): last section's pieces
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
            __builtin_amdgcn_s_barrier();
            if (MODE != 5) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int a = 0; a < 5; ++a)
                    acc[a * 4 + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[a], fa[b], acc[a * 4 + b], 0, 0, 0);
            if (MODE != 5) __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_s_barrier();
        }
        if (!grp) __builtin_amdgcn_s_barrier();
    }
    for (int it = 0; it < (MODE >= 4 ? 0 : iters); ++it) {
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

static char* g_src = nullptr;

template <int MODE, int NP = 0>
float run(float* out, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<MODE, NP><<<256, 512>>>(out, iters, g_src);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k<MODE, NP><<<256, 512>>>(out, iters, g_src);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / 5 * 1e3;
}

int main() {
    float* out; hipMalloc(&out, 4096);
    hipMalloc(&g_src, 64 << 20);
    hipMemset(g_src, 0, 64 << 20);
    const int iters = 2000;
    // per iteration per SIMD: 2 waves x 20 MFMA x 16 cycles = 640 cycles
    float t0 = run<0>(out, iters), t1 = run<1>(out, iters), t2 = run<2>(out, iters), t3 = run<3>(out, iters);
    float t4 = run<4>(out, iters), t5 = run<5>(out, iters);
    printf("reads+mfma %.1f us | mfma only %.1f us | reads only %.1f us | reads+mfma(AGPR acc) %.1f us\n", t0, t1, t2, t3);
    printf("ping-pong (setprio) %.1f us | ping-pong (no setprio) %.1f us\n", t4, t5);
    printf("ping-pong + DMA pieces per read section: 1: %.1f  2: %.1f  3: %.1f  4: %.1f us\n", run<6, 1>(out, iters),
           run<6, 2>(out, iters), run<6, 3>(out, iters), run<6, 4>(out, iters));
    printf("ideal mfma at 2.0 GHz: %.1f us\n", iters * 640 / 2.0e3);
    return 0;
}
