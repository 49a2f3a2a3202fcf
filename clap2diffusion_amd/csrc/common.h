// Shared device helpers for the gfx950 kernels of libc2d_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <type_traits>
#include <mutex>
#include "../../include/c2d.h"

typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define LDS_AS __attribute__((address_space(3)))



// Timing-ablation switches (C2D_GEMM_ABL / C2D_ATTN_ABL: skip the DMA, the MFMAs or
// the epilogue to attribute kernel time; wrong results by design) exist only in a
// bench build compiled with -DC2D_ENABLE_ABLATION (scripts/gpu_abl_tiles.sh).  In the
// production library every ablation test folds to a constant 0 and the environment
// variables are never read.
#ifdef C2D_ENABLE_ABLATION
#define C2D_ABL(x, bit) ((x) & (bit))
#else
#define C2D_ABL(x, bit) 0
#endif

namespace c2d {

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).  For loops whose
// body is too large for the unroller (which then leaves an accumulator array indexed
// by a run-time counter, i.e. in scratch memory): here every index is a constant.
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// thread-local last launch error, exposed as c2d_last_hip_error() (runtime.hip)
extern thread_local int g_last_hip_error;

// Tuning constants (A/B only; the defaults are the measured best).  Compile-time: an A/B
// candidate is a variant build (python -m clap2diffusion_amd.build --variant x --define
// C2D_TUNE_GN_FOLD=0, loaded through C2D_LIB), so the production library reads no
// environment variable and cannot be switched to another kernel or numerics at run time.
#ifndef C2D_TUNE_GEMM_MODE
#define C2D_TUNE_GEMM_MODE 0        // 2: register-staged kernels only
#endif
#ifndef C2D_TUNE_GEMM_KORDER
#define C2D_TUNE_GEMM_KORDER 1      // 3x3 K order: channel-block outer (1) / tap outer (0)
#endif
#ifndef C2D_TUNE_GEMM_LDSEPI
#define C2D_TUNE_GEMM_LDSEPI 1      // 0: direct 32x32 GEGLU epilogue
#endif
#ifndef C2D_TUNE_SPLITK_F16
#define C2D_TUNE_SPLITK_F16 0       // 1: split-K partials in fp16 (cancelling partials lose range / precision)
#endif
#ifndef C2D_TUNE_TAIL_SPLIT
#define C2D_TUNE_TAIL_SPLIT 1       // 0: no image split of a quantisation tail
#endif
#ifndef C2D_TUNE_PANEL_REGB
#define C2D_TUNE_PANEL_REGB 0       // 1: the K = 320 panel GEMM loads its weights into registers
#endif
#ifndef C2D_TUNE_PANEL_STAGGER
#define C2D_TUNE_PANEL_STAGGER 2    // panel GEMM: late start of waves 4-7, x 2048 cycles
#endif
#ifndef C2D_TUNE_PANEL_CARRY
#define C2D_TUNE_PANEL_CARRY 1      // K = 320 GEGLU panel GEMM runs each block's epilogue inside the next block's K loop
#endif
#ifndef C2D_TUNE_PANEL_PRIO
#define C2D_TUNE_PANEL_PRIO 1       // panel GEMM waves 4-7 at s_setprio 1
#endif
#ifndef C2D_TUNE_ATTN_NEGC
#define C2D_TUNE_ATTN_NEGC 1
#endif
#ifndef C2D_TUNE_ATTN_RES
#define C2D_TUNE_ATTN_RES 1
#endif
#ifndef C2D_TUNE_ATTN_W8
#define C2D_TUNE_ATTN_W8 1
#endif
#ifndef C2D_TUNE_ATTN_PP
#define C2D_TUNE_ATTN_PP 0
#endif
#ifndef C2D_TUNE_GN_BLOCKS
#define C2D_TUNE_GN_BLOCKS 512
#endif
#ifndef C2D_TUNE_GN_APPLY_BLOCKS
#define C2D_TUNE_GN_APPLY_BLOCKS 2048
#endif
#ifndef C2D_TUNE_GN_FUSED_HW
#define C2D_TUNE_GN_FUSED_HW 256
#endif
#ifndef C2D_TUNE_GN_FOLD
#define C2D_TUNE_GN_FOLD 1          // 0: partial + finalize + apply
#endif
#ifndef C2D_TUNE_GN_FOLD_CAP
#define C2D_TUNE_GN_FOLD_CAP 32     // most partial blocks per image on the fold path
#endif
#ifndef C2D_TUNE_GN_FOLD_APPLY_BLOCKS
#define C2D_TUNE_GN_FOLD_APPLY_BLOCKS 1024   // apply workgroups per launch (fold path, batches below 8 images)
#endif
struct Tuning {
    int gemm_mode, gemm_korder, gemm_lds_epi, splitk_f16, tail_split, panel_regb, panel_stagger;
    int attn_negc, attn_res, attn_w8, attn_pp;
    int gn_blocks, gn_apply_blocks, gn_fused_hw, gn_fold, gn_fold_cap, gn_fold_apply_blocks;
};
constexpr Tuning kTuning = {
    C2D_TUNE_GEMM_MODE, C2D_TUNE_GEMM_KORDER, C2D_TUNE_GEMM_LDSEPI, C2D_TUNE_SPLITK_F16, C2D_TUNE_TAIL_SPLIT,
    C2D_TUNE_PANEL_REGB, C2D_TUNE_PANEL_STAGGER,
    C2D_TUNE_ATTN_NEGC, C2D_TUNE_ATTN_RES, C2D_TUNE_ATTN_W8, C2D_TUNE_ATTN_PP,
    C2D_TUNE_GN_BLOCKS < 64 ? 512 : C2D_TUNE_GN_BLOCKS, C2D_TUNE_GN_APPLY_BLOCKS < 64 ? 2048 : C2D_TUNE_GN_APPLY_BLOCKS,
    C2D_TUNE_GN_FUSED_HW, C2D_TUNE_GN_FOLD, C2D_TUNE_GN_FOLD_CAP < 1 ? 32 : C2D_TUNE_GN_FOLD_CAP,
    C2D_TUNE_GN_FOLD_APPLY_BLOCKS < 64 ? 1024 : C2D_TUNE_GN_FOLD_APPLY_BLOCKS,
};
constexpr const Tuning& tuning() { return kTuning; }
// timing-ablation masks: C2D_GEMM_ABL / C2D_ATTN_ABL read from the environment in the
// -DC2D_ENABLE_ABLATION build only (runtime.hip); 0 in the production library
int ablation_gemm();
int ablation_attn();
// c2d_set_plan_override (tests / sweeps): 0 = the planner decides
int plan_override_tile();
int plan_override_split();
constexpr int kMaxDevices = 64;
int current_device();

// The per-device kernel table: kernels that declare more than the default 64 KiB of
// dynamic LDS get hipFuncAttributeMaxDynamicSharedMemorySize once per (kernel, device),
// under one std::once_flag per device for each kernel instantiation K (thread-safe on a
// first concurrent call from several host threads, and per device on multi-GPU hosts).
template <auto K>
inline void ensure_lds(int bytes) {
    static std::once_flag once[kMaxDevices];
    std::call_once(once[current_device()], [bytes] {
        (void)hipFuncSetAttribute((const void*)K, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    });
}

inline int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_last_hip_error = (int)e;
        return C2D_E_HIP;
    }
    return C2D_OK;
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
// x * sigmoid(k x): SiLU (k = 1) and quick_gelu (k = 1.702, CLIP text MLP)
__device__ __forceinline__ float sigmoid_lin(float x, float k) { return x / (1.0f + __expf(-k * x)); }
// erf-form GELU (torch's default, what diffusers' GEGLU / HTSAT's MLP use) with a
// branch-free erf: Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 -- far below the
// fp16 rounding of every output it feeds -- in ~14 VALU ops (one rcp, one exp)
// instead of the library erff's piecewise branches (the GEGLU epilogue runs it
// on 84M elements per level-0 call).
__device__ __forceinline__ float erf_as(float x) {
    const float z = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float e = 1.0f - p * t * __expf(-z * z);
    return copysignf(e, x);
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.0f + erf_as(x * 0.70710678118654752f)); }

// GELU of the GEGLU epilogues (gelu_f stays for C2D_ACT_GELU): x * sigmoid(z), z = x' (a + b x'^2 + c x'^4), x' = x
// clamped to [-8, 8] (z monotone there; sigmoid(z(+-8)) is 1 / 0 to 1e-12).  Coefficients fitted
// (near-minimax) to the erf form 0.5 x (1 + erf(x / sqrt 2)) diffusers' GEGLU uses: max
// |error| 3.4e-5 over the real line, below the fp16 rounding of every GEGLU output above
// 0.07 in magnitude; 7 VALU + 2 transcendental issue slots against ~17 + 2 for the
// Abramowitz-Stegun erf (gelu_f), the op count the carried epilogue hides under the MFMAs.
// log2(e) is folded into the coefficients (exp2 on the hardware unit).
__device__ __forceinline__ float gelu_sig(float x) {
    const float xc = __builtin_amdgcn_fmed3f(x, -8.0f, 8.0f);
    const float x2 = xc * xc;
    const float z = xc * fmaf(fmaf(-0.0009763994f, x2, 0.10652431f), x2, 2.3013635f);   // (a, b, c) * log2 e
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z));
}
// h * gelu_sig(g) on two lanes' worth of values at once: the polynomial and the products on
// packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two results per issue), the clamp,
// exp2 and rcp per element -- same formula and coefficients as gelu_sig
__device__ __forceinline__ f32x2 geglu2(f32x2 h, f32x2 g) {
    const f32x2 xc = {__builtin_amdgcn_fmed3f(g.x, -8.0f, 8.0f), __builtin_amdgcn_fmed3f(g.y, -8.0f, 8.0f)};
    const f32x2 x2 = xc * xc;
    f32x2 q = __builtin_elementwise_fma(x2, (f32x2){0.0009763994f, 0.0009763994f},
                                        (f32x2){-0.10652431f, -0.10652431f});
    q = __builtin_elementwise_fma(q, x2, (f32x2){-2.3013635f, -2.3013635f});
    const f32x2 nz = xc * q;   // -z
    f32x2 e = {__builtin_amdgcn_exp2f(nz.x), __builtin_amdgcn_exp2f(nz.y)};
    e = e + (f32x2){1.0f, 1.0f};
    const f32x2 hg = h * g;
    return hg * (f32x2){__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y)};
}


// bijective XCD-aware block remap (8 XCDs, round-robin dispatch): blocks that
// land on one XCD get a contiguous range of tile ids so they share L2 panels.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg >> 3, r = nwg & 7;
    const int xcd = bid & 7, local = bid >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// a kernel-argument pointer the compiler can prove wave-uniform (two readfirstlane
// halves): keeps it in SGPRs across loops instead of re-loading it from the
// kernarg segment behind an s_waitcnt every iteration
__device__ __forceinline__ const char* uniform_ptr(const void* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const char*)(((uint64_t)hi << 32) | lo);
}

// buffer resource over [base, base + bytes): loads / DMA pieces past num_records read zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

}  // namespace c2d
