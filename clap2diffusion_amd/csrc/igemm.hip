// Implicit-GEMM convolution / linear kernel for gfx950 (MFMA f32_16x16x32_f16).
//
//   out[m, j] = act(sum_k A[m, k] W[j, k] + bias[j]) + temb[n(m), j] + resid[m, j]
//
// A = on-the-fly im2col of an NHWC fp16 input (optionally two channel sources,
// i.e. the UNet skip concat, and optionally a nearest-x2 upsampled view), with a
// fused prologue (GroupNorm affine [+SiLU], LayerNorm, or SiLU) applied to the
// in-bounds elements only, so zero padding stays zero after normalisation as in
// torch (conv pads the *normalised* tensor).  W = packed [cout][kpad] fp16.
//
// Tiling: BM x BN block tile (128x128 or 64x64), BK = 64, 256 threads = 4 waves
// in 2x2, each wave (BM/2)x(BN/2) of 16x16 MFMA tiles.  The MFMA computes the
// transposed product D^T = W . A^T so every lane ends with 4 consecutive output
// columns of one row: the epilogue stores 8-byte row segments straight to HBM.
// A and B tiles are register-staged (load early, transform, ds_write_b128 late)
// into a double-buffered, XOR-swizzled LDS image: one barrier per K step.
#include "common.h"
#include <stdlib.h>
#include <type_traits>

// 0 = A/B builds only: the 32x32 tiles 25 / 1 in place of the ping-pong 40 / 41 defaults
#ifndef C2D_PP16_DEFAULT
#define C2D_PP16_DEFAULT 1
#endif

// The library compiles this file once per kernel family (build.py: -DC2D_IGEMM_PART=k)
// so the families build in parallel: 0 = host API, planner, register-staged kernels and
// the split-K combine; 1 = ping-pong 16x16x32 tiles; 2 = 32x32x16 tiles; 3 = 16x16x32
// LDS-DMA tiles; 4 = the panel GEMM.  Undefined (-1) = everything in one object.
#ifndef C2D_IGEMM_PART
#define C2D_IGEMM_PART -1
#endif
#define C2D_PART(k) (C2D_IGEMM_PART < 0 || C2D_IGEMM_PART == (k))

namespace c2d {

enum AMode { AM_1X1 = 0, AM_3X3_FAST = 1, AM_3X3_GEN = 2 };

struct IgemmParams {
    const f16* src0; const f16* src1; int c0, c1, cin;
    int n, h, w, oh, ow, stride, up, pad;
    int vh, vw;  // virtual (possibly upsampled) input size
    const f16* wt; int cout, kpad, ktot;
    int pro, pro_silu;
    const float* pro_a; const float* pro_b; const float* gamma; const float* beta;
    const float* bias; int act;
    const f16* temb; int temb_ld;
    const f16* resid; int resid_ld;
    f16* out; int out_ld;
    int M;       // rows = n*oh*ow
    int gx, gy;  // tiles along cout / M
    int ksplit;  // K slices per output tile (DMA path; 1 = no split)
    int nkt;     // K steps per slice
    float* ws;   // split-K partials [ksplit][M][cout]: fp32, or fp16 when slab16
    int slab16;  // split-K partials stored as fp16 (C2D_TUNE_SPLITK_F16): half the slab write + combine read
    int abl;     // timing ablation bits (C2D_GEMM_ABL; 0 in production)
    int lds_epi; // 32x32 kernels: 1 = LDS-staged epilogue (C2D_TUNE_GEMM_LDSEPI or alignment), 0 = direct
    int cmajor;  // DMA 3x3 kernels: K steps channel-block-outer / tap-inner (C2D_TUNE_GEMM_KORDER, default 1)
    float pro_eps;   // C2D_PRO_LNFOLD: LayerNorm eps
    float* gn_mom;   // GroupNorm moments of the output ({mean, M2} per (image, tile, group)) or NULL (row-ring tiles only)
    int gn_cpg;      // channels per group of gn_mom
};

// one accumulator quad of K slice `slice` into the split-K workspace, fp32 or rounded to fp16
__device__ __forceinline__ void store_partial(const IgemmParams& p, int slice, int m, int j, const f32x4& v) {
    const size_t off = ((size_t)slice * p.M + m) * p.cout + j;
    if (p.slab16) {
        const f16x4 h = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
        *reinterpret_cast<f16x4*>(reinterpret_cast<f16*>(p.ws) + off) = h;
    } else {
        *reinterpret_cast<f32x4*>(p.ws + off) = v;
    }
}

}  // namespace c2d
#include "epilogue.h"
namespace c2d {

// byte offset of 16-byte chunk `c` (0..7) of `row` in a [rows][64] fp16 LDS tile
__device__ __forceinline__ int lds_off(int row, int c) { return row * 128 + ((c ^ ((row >> 1) & 7)) << 4); }

template <int BM>
struct RowInfo {
    int n[BM / 32], iy[BM / 32], ix[BM / 32];
    bool ok[BM / 32];
};

__device__ __forceinline__ f16x8 zero8() {
    f16x8 z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = (f16)0.f;
    return z;
}

// Load one 16-B chunk of A (8 channels) for output row described by (n, iy, ix)
template <int AMODE>
__device__ __forceinline__ f16x8 load_a_chunk(const IgemmParams& p, int n, int iy0, int ix0, bool rok,
                                              int k, int tap_fast, int cbase_fast, int cc, int& cout_c,
                                              bool& valid) {
    int c, ky, kx;
    if (AMODE == AM_1X1) {
        c = k; ky = 0; kx = 0;
        valid = rok && (c < p.cin);
    } else if (AMODE == AM_3X3_FAST) {
        c = cbase_fast + cc * 8;
        ky = tap_fast / 3; kx = tap_fast - ky * 3;
        valid = rok;
    } else {
        int tap = k / p.cin;
        c = k - tap * p.cin;
        ky = tap / 3; kx = tap - ky * 3;
        valid = rok && (tap < 9);
    }
    int iy = iy0 + ky, ix = ix0 + kx;
    valid = valid && iy >= 0 && iy < p.vh && ix >= 0 && ix < p.vw;
    cout_c = c;
    if (!valid) return zero8();
    if (p.up) { iy >>= 1; ix >>= 1; }
    size_t pix = ((size_t)n * p.h + iy) * p.w + ix;
    const f16* ptr = (c < p.c0) ? (p.src0 + pix * p.c0 + c) : (p.src1 + pix * p.c1 + (c - p.c0));
    return *reinterpret_cast<const f16x8*>(ptr);
}

__device__ __forceinline__ f16x8 apply_pro(const IgemmParams& p, f16x8 v, int n, int m, int c) {
    if (p.pro == C2D_PRO_GN) {
        const float4* sc = reinterpret_cast<const float4*>(p.pro_a + (size_t)n * p.cin + c);
        const float4* sh = reinterpret_cast<const float4*>(p.pro_b + (size_t)n * p.cin + c);
        float4 s0 = sc[0], s1 = sc[1], h0 = sh[0], h1 = sh[1];
        float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        float hh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float y = (float)v[i] * s[i] + hh[i];
            if (p.pro_silu) y = silu_f(y);
            v[i] = (f16)y;
        }
    } else if (p.pro == C2D_PRO_LN) {
        float2 st = *reinterpret_cast<const float2*>(p.pro_a + (size_t)m * 2);
        const float4* g = reinterpret_cast<const float4*>(p.gamma + c);
        const float4* b = reinterpret_cast<const float4*>(p.beta + c);
        float4 g0 = g[0], g1 = g[1], b0 = b[0], b1 = b[1];
        float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
        float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (f16)(((float)v[i] - st.x) * st.y * gg[i] + bb[i]);
    } else if (p.pro == C2D_PRO_SILU) {
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (f16)silu_f((float)v[i]);
    }
    return v;
}

// ---- epilogue: lane holds out[row mrow0 + 16 b + (lane&15)][cols ncol0 + 16 a + 4 (lane>>4) .. +3]
// All operand loads (bias, temb, residual) are issued first from clamped, always
// valid addresses, then the math, then the stores: no load waits behind a store
// (out may alias resid for in-place residual adds; every element is read before
// it is written by the same lane, so that stays correct).
template <int TM, int TN>
__device__ __forceinline__ void epilogue_tiles(const IgemmParams& p, f32x4 (&acc)[TN][TM], int mrow0, int ncol0,
                                               int lane) {
    const int hw = p.oh * p.ow;
    const int lr = lane & 15, lc = 4 * (lane >> 4);
    int mrow[TM], nimg[TM];
    bool mok[TM];
#pragma unroll
    for (int b = 0; b < TM; ++b) {
        const int m = mrow0 + b * 16 + lr;
        mok[b] = m < p.M;
        mrow[b] = mok[b] ? m : p.M - 1;
        nimg[b] = mrow[b] / hw;
    }
    if (p.act != C2D_ACT_GEGLU) {
        int col[TN];
        bool cok[TN];
        float4 bv[TN];
#pragma unroll
        for (int a = 0; a < TN; ++a) {
            const int j = ncol0 + a * 16 + lc;
            cok[a] = j < p.cout;
            col[a] = cok[a] ? j : 0;
            bv[a] = p.bias ? *reinterpret_cast<const float4*>(p.bias + col[a]) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        f16x4 rv[TM][TN], tv[TM][TN];
        if (p.resid) {
#pragma unroll
            for (int b = 0; b < TM; ++b)
#pragma unroll
                for (int a = 0; a < TN; ++a)
                    rv[b][a] = *reinterpret_cast<const f16x4*>(p.resid + (size_t)mrow[b] * p.resid_ld + col[a]);
        }
        if (p.temb) {
#pragma unroll
            for (int b = 0; b < TM; ++b)
#pragma unroll
                for (int a = 0; a < TN; ++a)
                    tv[b][a] = *reinterpret_cast<const f16x4*>(p.temb + (size_t)nimg[b] * p.temb_ld + col[a]);
        }
#pragma unroll
        for (int b = 0; b < TM; ++b) {
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                float v[4] = {acc[a][b][0] + bv[a].x, acc[a][b][1] + bv[a].y, acc[a][b][2] + bv[a].z,
                              acc[a][b][3] + bv[a].w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (p.act == C2D_ACT_GELU) v[r] = gelu_f(v[r]);
                    else if (p.act == C2D_ACT_RELU) v[r] = fmaxf(v[r], 0.f);
                    else if (p.act == C2D_ACT_SILU) v[r] = silu_f(v[r]);
                    else if (p.act == C2D_ACT_QUICK_GELU) v[r] = sigmoid_lin(v[r], 1.702f);
                    if (p.temb) v[r] += (float)tv[b][a][r];
                    if (p.resid) v[r] += (float)rv[b][a][r];
                }
                f16x4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = (f16)v[r];
                if (mok[b] && cok[a]) *reinterpret_cast<f16x4*>(p.out + (size_t)mrow[b] * p.out_ld + col[a]) = o;
            }
        }
    } else {
        // packed rows: [16 h | 16 g] per 32-row block -> 16 output features
        constexpr int TP = TN / 2;
        int jo[TP], jh[TP];
        bool cok[TP];
        float4 bh[TP], bg[TP];
#pragma unroll
        for (int q = 0; q < TP; ++q) {
            const int jp = ncol0 + 2 * q * 16;
            cok[q] = jp < p.cout;
            const int jpc = cok[q] ? jp : 0;
            jo[q] = (jpc >> 1) + lc;
            jh[q] = jpc + lc;
            bh[q] = p.bias ? *reinterpret_cast<const float4*>(p.bias + jh[q]) : make_float4(0.f, 0.f, 0.f, 0.f);
            bg[q] = p.bias ? *reinterpret_cast<const float4*>(p.bias + jh[q] + 16) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        f16x4 rv[TM][TP];
        if (p.resid) {
#pragma unroll
            for (int b = 0; b < TM; ++b)
#pragma unroll
                for (int q = 0; q < TP; ++q)
                    rv[b][q] = *reinterpret_cast<const f16x4*>(p.resid + (size_t)mrow[b] * p.resid_ld + jo[q]);
        }
#pragma unroll
        for (int b = 0; b < TM; ++b) {
#pragma unroll
            for (int q = 0; q < TP; ++q) {
                const f32x4 h4 = acc[2 * q][b], g4 = acc[2 * q + 1][b];
                const float hb[4] = {bh[q].x, bh[q].y, bh[q].z, bh[q].w}, gb[4] = {bg[q].x, bg[q].y, bg[q].z, bg[q].w};
                f16x4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = (h4[r] + hb[r]) * gelu_sig(g4[r] + gb[r]);
                    if (p.resid) v += (float)rv[b][q][r];
                    o[r] = (f16)v;
                }
                if (mok[b] && cok[q]) *reinterpret_cast<f16x4*>(p.out + (size_t)mrow[b] * p.out_ld + jo[q]) = o;
            }
        }
    }
}

template <int BM, int BN>
__device__ __forceinline__ void epilogue(const IgemmParams& p, f32x4 (&acc)[BN / 32][BM / 32], int m0, int n0, int wm,
                                         int wn, int lane) {
    epilogue_tiles<BM / 32, BN / 32>(p, acc, m0 + wm * (BM / 2), n0 + wn * (BN / 2), lane);
}

// per-wave 64x64 tile epilogue
__device__ __forceinline__ void epilogue_w64(const IgemmParams& p, f32x4 (&acc)[4][4], int mw0, int nw0, int lane) {
    epilogue_tiles<4, 4>(p, acc, mw0, nw0, lane);
}

template <int BM, int BN, int AMODE>
__global__ void __launch_bounds__(256) igemm_kernel(IgemmParams p) {
    constexpr int TM = BM / 32;  // 16-row MFMA tiles per wave along M
    constexpr int TN = BN / 32;  // along N
    constexpr int ACH = BM / 32; // A chunks per thread per K step
    constexpr int BCH = BN / 32;
    constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int tile = xcd_remap(blockIdx.x, p.gx * p.gy);
    const int mt = tile / p.gx, nt = tile - mt * p.gx;
    const int m0 = mt * BM, n0 = nt * BN;

    // per-thread staging rows (fixed across K): chunk cc, rows tid/8 + 32 i
    const int cc = tid & 7;
    const int hw = p.oh * p.ow;
    int a_n[ACH], a_iy[ACH], a_ix[ACH], a_m[ACH];
    bool a_ok[ACH];
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
        int m = m0 + (tid >> 3) + 32 * i;
        a_m[i] = m;
        a_ok[i] = m < p.M;
        int mm = a_ok[i] ? m : 0;
        int nn = mm / hw, r = mm - nn * hw;
        int oy = r / p.ow, ox = r - oy * p.ow;
        a_n[i] = nn;
        a_iy[i] = oy * p.stride - p.pad;
        a_ix[i] = ox * p.stride - p.pad;
    }
    const f16* b_ptr[BCH];
    bool b_ok[BCH];
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
        int j = n0 + (tid >> 3) + 32 * i;
        b_ok[i] = j < p.cout;
        b_ptr[i] = p.wt + (size_t)(b_ok[i] ? j : 0) * p.kpad + cc * 8;
    }

    f32x4 acc[TN][TM];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

    f16x8 ra[ACH], rb[BCH];
    int rc[ACH];
    bool rv[ACH];
    const int nk = p.kpad / 64;

    auto gload = [&](int kt) {
        const int k0 = kt * 64;
        int tap = 0, cbase = 0;
        if (AMODE == AM_3X3_FAST) { tap = k0 / p.cin; cbase = k0 - tap * p.cin; }
#pragma unroll
        for (int i = 0; i < ACH; ++i)
            ra[i] = load_a_chunk<AMODE>(p, a_n[i], a_iy[i], a_ix[i], a_ok[i], k0 + cc * 8, tap, cbase, cc, rc[i], rv[i]);
#pragma unroll
        for (int i = 0; i < BCH; ++i)
            rb[i] = b_ok[i] ? *reinterpret_cast<const f16x8*>(b_ptr[i] + k0) : zero8();
    };
    auto swrite = [&](int buf) {
        char* As = smem + buf * (A_BYTES + B_BYTES);
        char* Bs = As + A_BYTES;
#pragma unroll
        for (int i = 0; i < ACH; ++i) {
            f16x8 v = ra[i];
            if (p.pro != C2D_PRO_NONE && rv[i]) v = apply_pro(p, v, a_n[i], a_m[i], rc[i]);
            int row = (tid >> 3) + 32 * i;
            *reinterpret_cast<f16x8*>(As + lds_off(row, cc)) = v;
        }
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            int row = (tid >> 3) + 32 * i;
            *reinterpret_cast<f16x8*>(Bs + lds_off(row, cc)) = rb[i];
        }
    };

    gload(0);
    swrite(0);
    __syncthreads();

    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload(kt + 1);
        const char* As = smem + buf * (A_BYTES + B_BYTES);
        const char* Bs = As + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = kk * 4 + (lane >> 4);
            f16x8 fa[TM], fb[TN];
#pragma unroll
            for (int t = 0; t < TM; ++t) {
                int row = wm * (BM / 2) + t * 16 + (lane & 15);
                fa[t] = *reinterpret_cast<const f16x8*>(As + lds_off(row, ch));
            }
#pragma unroll
            for (int t = 0; t < TN; ++t) {
                int row = wn * (BN / 2) + t * 16 + (lane & 15);
                fb[t] = *reinterpret_cast<const f16x8*>(Bs + lds_off(row, ch));
            }
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[a], fa[b], acc[a][b], 0, 0, 0);
        }
        if (kt + 1 < nk) swrite(buf ^ 1);
        __syncthreads();
    }

    epilogue<BM, BN>(p, acc, m0, n0, wm, wn, lane);
}


// ---------------------------------------------------------------------------
// LDS-DMA implicit-GEMM kernels (no prologue).
//
// A and B tiles go HBM -> LDS with buffer_load_dwordx4 ... lds (16 B per lane,
// one 1-KiB wave instruction per 8 tile rows) into a STAGES-deep ring; stage
// kt+S-1 is issued right after the barrier that proves stage kt landed, so S-1
// K steps of loads are in flight behind the MFMAs.  Waits are counted (vmcnt =
// pieces per stage x stages left in flight) and the barrier is a raw s_barrier,
// so nothing drains the ring inside the loop.  The LDS image is lane-linear: the
// XOR bank swizzle goes on the per-lane SOURCE chunk (slot s of row r fetches
// logical chunk s ^ f(r)) and is undone on the read (lds_off).
//
// Addressing: every K step is one (tap, channel block) pair, so the per-step
// part of the source address (tap displacement, channel base, which concat
// source) is wave-uniform and goes into the buffer descriptor's base; the lane
// keeps a precomputed 32-bit byte offset per staged row and a 9-bit in-bounds
// mask over the 3x3 taps.  Halo / tail lanes get an offset past num_records, and
// the buffer unit's range check returns zeros for them -- no zero page, no
// 64-bit address math.  Weight rows past cout are likewise out of range.
// Requires c0 % 64 == 0 when two sources are used (a 64-wide K step never
// straddles the concat seam) and no nearest-x2 view.
typedef __attribute__((address_space(3))) void* lptr_t;
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ void wait_vmcnt_le(int n) {
    // s_waitcnt simm16 (gfx9 family): vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt_hi[15:14]
#define C2D_WAITVM(N) __builtin_amdgcn_s_waitcnt(((N) & 15) | (7 << 4) | (15 << 8) | (((N) >> 4) << 14))
    switch (n) {
        case 4: C2D_WAITVM(4); break;
        case 6: C2D_WAITVM(6); break;
        case 8: C2D_WAITVM(8); break;
        case 12: C2D_WAITVM(12); break;
        case 16: C2D_WAITVM(16); break;
        default: C2D_WAITVM(0); break;
    }
#undef C2D_WAITVM
}


// one 1-KiB DMA piece: lane l's 16 bytes at rsrc.base + off land at lds + 16 l
__device__ __forceinline__ void dma_piece(__amdgpu_buffer_rsrc_t r, char* lds, unsigned off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)lds, 16, off, 0, 0, 0);
}

// TM x TN 16x16 tiles of a per-wave accumulator, written in row chunks of <= 4
// tiles so the hoisted epilogue operands stay within the register budget.
template <int TM, int TN>
__device__ __forceinline__ void epilogue_chunked(const IgemmParams& p, f32x4 (&acc)[TN][TM], int mrow0, int ncol0,
                                                 int lane) {
    constexpr int MC = TM < 4 ? TM : 4;
#pragma unroll
    for (int b0 = 0; b0 < TM; b0 += MC) {
        f32x4 sub[TN][MC];
#pragma unroll
        for (int a = 0; a < TN; ++a)
#pragma unroll
            for (int b = 0; b < MC; ++b) sub[a][b] = acc[a][b0 + b];
        epilogue_tiles<MC, TN>(p, sub, mrow0 + b0 * 16, ncol0, lane);
    }
}

// KG > 1: intra-workgroup split-K.  KG groups of WM x WN waves share the output tile, group g
// walking its own contiguous share of the block's K steps through its own STAGES-slot ring;
// after the loop groups 1 .. KG-1 leave their raw accumulators in LDS (lane-linear, fixed
// order) and exit, group 0 adds them and runs the epilogue (or the split-K slab store).  Two
// waves per SIMD on the under-filled grids (level-2 / level-3 GEMMs: one 4-wave tile per CU)
// with no fp32 slab traffic and no combine launch.
template <int WM, int WN, int TM, int TN, int STAGES, int KS, int KG = 1>
__global__ void __launch_bounds__(64 * WM * WN * KG) igemm_dma_kernel(IgemmParams p) {
    constexpr int NW = WM * WN;
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW);   // DMA pieces per wave per stage
    constexpr int PER = AI + BI;
    constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
    static_assert(AI * 8 * NW == BM && BI * 8 * NW == BN, "tile / wave mismatch");
    extern __shared__ __attribute__((aligned(16))) char smem_all[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kg = wave_all / NW, wave = wave_all - kg * NW;   // K group, wave within the group
    char* const smem = smem_all + (KG > 1 ? kg * STAGES * STAGE : 0);
    const int wm = wave / WN, wn = wave - (wave / WN) * WN;
    // block -> (output tile, K slice); the remap keeps a tile's slices on one XCD
    const int bid = xcd_remap(blockIdx.x, p.gx * p.gy * p.ksplit);
    const int tile = bid / p.ksplit, slice = bid - tile * p.ksplit;
    const int mt = tile / p.gx, nt = tile - mt * p.gx;
    const int m0 = mt * BM, n0 = nt * BN;
    const int lrow = lane >> 3, slot = lane & 7;
    const int hw = p.oh * p.ow;
    const bool two = p.c1 > 0;
    const int pshift = KS == 3 ? p.w + 1 : 0;

    // ---- per staged A row: byte offsets in each source + tap mask
    unsigned a_off0[AI], a_off1[AI], a_mask[AI];
    int a_ch[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
        const int row = (wave * AI + i) * 8 + lrow;
        const int m = m0 + row;
        const int mm = m < p.M ? m : 0;
        const int nn = mm / hw, r = mm - nn * hw;
        const int oy = r / p.ow, ox = r - oy * p.ow;
        const int iy0 = oy * p.stride - p.pad, ix0 = ox * p.stride - p.pad;
        unsigned mask = 0;
        if (m < p.M) {
#pragma unroll
            for (int ky = 0; ky < KS; ++ky)
#pragma unroll
                for (int kx = 0; kx < KS; ++kx)
                    if (iy0 + ky >= 0 && iy0 + ky < p.h && ix0 + kx >= 0 && ix0 + kx < p.w) mask |= 1u << (ky * KS + kx);
        }
        // window origin, biased by pshift pixels so every offset is >= 0 (the halo
        // origin of the first pixel is -(w+1)); the descriptor base is biased back
        const int pix0 = (nn * p.h + iy0) * p.w + ix0 + pshift;
        a_ch[i] = (slot ^ ((row >> 1) & 7)) * 8;
        a_off0[i] = (unsigned)(2 * (pix0 * p.c0 + a_ch[i]));
        a_off1[i] = (unsigned)(2 * (pix0 * p.c1 + a_ch[i]));
        a_mask[i] = mask;
    }
    unsigned b_off[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
        const int row = (wave * BI + i) * 8 + lrow;
        const int j = n0 + row;
        b_off[i] = (j < p.cout) ? (unsigned)(2 * (j * p.kpad + (slot ^ ((row >> 1) & 7)) * 8)) : kOOB;
    }
    const size_t npix = (size_t)p.n * p.h * p.w;
    const unsigned bytes0 = (unsigned)(npix * p.c0 * 2), bytes1 = (unsigned)(npix * p.c1 * 2);
    const unsigned wbytes = (unsigned)((size_t)p.cout * p.kpad * 2);
    const bool ctail = (p.cin & 63) != 0;

    const int nk_all = p.kpad / 64;
    const int kb0 = slice * p.nkt, ke0 = min(nk_all, kb0 + p.nkt);   // this block's K steps [kb0, ke0)
    const int kper = (ke0 - kb0 + KG - 1) / KG;                      // steps per K group (the loop count)
    const int kb = min(ke0, kb0 + kg * kper), ke = min(ke0, kb + kper);   // this group's share
    const char* u_src0 = uniform_ptr(p.src0);
    const char* u_src1 = uniform_ptr(p.src1);
    const char* u_wt = uniform_ptr(p.wt);
    // (tap, channel block) of the next issue; the packed weight column is tap * cin + cbase
    int tap = 0, cbase = kb * 64;
    if (KS == 3) {
        if (p.cmajor) { tap = kb % 9; cbase = (kb / 9) * 64; }
        else { tap = cbase / p.cin; cbase -= tap * p.cin; }
    }
    auto issue = [&](int kt, int buf) {
        (void)kt;
        const int k0 = tap * p.cin + cbase;
        const int ky = tap / 3, kx = tap - (tap / 3) * 3;
        const bool use1 = two && cbase >= p.c0;
        const int cs = use1 ? p.c1 : p.c0;
        const unsigned sterm = 2u * (unsigned)((KS == 3 ? (ky * p.w + kx) * cs : 0) + (use1 ? cbase - p.c0 : cbase));
        const char* sb = use1 ? u_src1 : u_src0;
        const unsigned bias = 2u * (unsigned)(pshift * cs);
        const unsigned sbytes = use1 ? bytes1 : bytes0;
        const __amdgpu_buffer_rsrc_t ra = make_rsrc(sb + sterm - bias, sbytes + bias - sterm);
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(u_wt + 2 * k0, wbytes - 2 * k0);
        const int lim = p.cin - cbase;                              // only binds on a channel tail
        char* base = smem + buf * STAGE;
#pragma unroll
        for (int i = 0; i < AI; ++i) {
            // branch-free: a dropped tap / channel tail pushes the offset past num_records
            unsigned ok = (a_mask[i] >> tap) & 1u;
            if (ctail) ok &= (unsigned)(a_ch[i] < lim);
            const unsigned off = (use1 ? a_off1[i] : a_off0[i]) | ((ok - 1u) & kOOB);
            dma_piece(ra, base + (wave * AI + i) * 1024, off);
        }
#pragma unroll
        for (int i = 0; i < BI; ++i)
            dma_piece(rb, base + A_BYTES + (wave * BI + i) * 1024, b_off[i]);
        if (KS == 3 && p.cmajor) {                                 // taps inner
            if (++tap == 9) { tap = 0; cbase += 64; }
        } else {                                                   // packed K order
            cbase += 64;
            if (KS == 3 && cbase >= p.cin) { cbase = 0; ++tap; }
        }
    };

    // ---- fragment read offsets: tile t of this wave = base + t * 2 KiB (the swizzle
    // depends only on row bits 1..3, i.e. on the lane)
    int fa0[2], fb0[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
        const int l = lds_off(lane & 15, kk * 4 + (lane >> 4));
        fa0[kk] = wm * TM * 2048 + l;
        fb0[kk] = A_BYTES + wn * TN * 2048 + l;
    }

    f32x4 acc[TN][TM];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int s0 = 0; s0 < STAGES - 1; ++s0)
        if (kb + s0 < ke) issue(kb + s0, s0);
    int rd = 0, wr = STAGES - 1;
    // every group runs kper trips (the barriers are workgroup-wide); a group with fewer steps
    // (the last share of an odd count) idles through its surplus trips
    const int kend = KG > 1 ? kb + kper : ke;
    for (int kt = kb; kt < kend; ++kt) {
        if (kt + STAGES - 2 < ke) wait_vmcnt_le(PER * (STAGES - 2));
        else wait_vmcnt_le(0);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        // p.abl (timing ablation only, C2D_GEMM_ABL): bit 0 skips the DMA after the
        // prologue stages, bit 1 skips the MFMAs (fragments still read and kept live)
        if (kt + STAGES - 1 < ke && !(C2D_ABL(p.abl, 1))) issue(kt + STAGES - 1, wr);
        const char* S = smem + rd * STAGE;
        if (KG > 1 && kt >= ke) continue;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            f16x8 fa[TM], fb[TN];
#pragma unroll
            for (int t = 0; t < TN; ++t) fb[t] = *reinterpret_cast<const f16x8*>(S + fb0[kk] + t * 2048);
#pragma unroll
            for (int t = 0; t < TM; ++t) fa[t] = *reinterpret_cast<const f16x8*>(S + fa0[kk] + t * 2048);
            if (C2D_ABL(p.abl, 2)) {
#pragma unroll
                for (int t = 0; t < TN; ++t) asm volatile("" :: "v"(fb[t]));
#pragma unroll
                for (int t = 0; t < TM; ++t) asm volatile("" :: "v"(fa[t]));
                continue;
            }
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int b = 0; b < TM; ++b)
#pragma unroll
                for (int a = 0; a < TN; ++a)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[a], fa[b], acc[a][b], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        rd = (rd + 1 == STAGES) ? 0 : rd + 1;
        wr = (wr + 1 == STAGES) ? 0 : wr + 1;
    }
    if constexpr (KG > 1) {
        // groups 1 .. KG-1 -> LDS (above the epilogue images), group 0 adds them in group order
        constexpr int EPI = NW * 16 * (TM < 2 ? TM : 2) * (TN * 16 + 4) * 4;
        constexpr int RED = (EPI + 1023) / 1024 * 1024;
        f32x4* red = reinterpret_cast<f32x4*>(smem_all + RED);
        __syncthreads();   // every group is done with its ring
        if (kg > 0) {
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b)
                    red[((((kg - 1) * NW + wave) * TN + a) * TM + b) * 64 + lane] = acc[a][b];
        }
        __syncthreads();
        if (kg > 0) return;   // s_barrier waits only on the surviving waves from here on
#pragma unroll
        for (int g = 1; g < KG; ++g)
#pragma unroll
            for (int a = 0; a < TN; ++a)
#pragma unroll
                for (int b = 0; b < TM; ++b) acc[a][b] += red[((((g - 1) * NW + wave) * TN + a) * TM + b) * 64 + lane];
    }
    if (p.ksplit > 1) {
        // raw fp32 partial sums; bias / act / temb / residual go in splitk_reduce_kernel
        const int mw0 = m0 + wm * TM * 16, nw0 = n0 + wn * TN * 16;
#pragma unroll
        for (int b = 0; b < TM; ++b) {
            const int m = mw0 + b * 16 + (lane & 15);
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                const int j = nw0 + a * 16 + 4 * (lane >> 4);
                if (m < p.M && j < p.cout) store_partial(p, slice, m, j, acc[a][b]);
            }
        }
        return;
    }
    // LDS-staged epilogue (epilogue.h): passes of up to 32 rows of fp32 per wave image,
    // the bias added as the accumulators are written
    __syncthreads();
    {
        constexpr int PITCHF = TN * 16 + 4;
        constexpr int RB = TM < 2 ? TM : 2;                  // 16-row tiles per image
        float* img = reinterpret_cast<float*>(smem) + wave * 16 * RB * PITCHF;
        const int mw0 = m0 + wm * TM * 16, nw0 = n0 + wn * TN * 16;
        static_for<0, TM / RB>([&](auto pass) __attribute__((always_inline)) {
            constexpr int b0 = RB * decltype(pass)::value;
            epi_pass<RB * 16, TN * 16, false>(p, img, PITCHF, mw0 + b0 * 16, nw0, lane, [&]() __attribute__((always_inline)) {
                f32x4 bv[TN];   // per pass (an L1 hit after the first): fewer registers held across passes
#pragma unroll
                for (int a = 0; a < TN; ++a) bv[a] = bias4(p, nw0 + a * 16 + 4 * (lane >> 4));
#pragma unroll
                for (int bb = 0; bb < RB; ++bb)
#pragma unroll
                    for (int a = 0; a < TN; ++a)
                        *reinterpret_cast<f32x4*>(img + (bb * 16 + (lane & 15)) * PITCHF + a * 16 + 4 * (lane >> 4)) =
                            acc[a][b0 + bb] + bv[a];
            });
        });
    }
}

#if C2D_PART(0)
// split-K combine + epilogue: out[m, j..j+3] = act(sum_s ws[s][m][j..] + bias) + temb + resid
// (same operation order as epilogue_tiles; slices summed in fixed order s = 0, 1, ...).
// KS > 0: the slice count is a compile-time constant and every slab load of an output
// quad is issued before the first add -- the runtime-count loop waited vmcnt(0) after
// each slab load, ks dependent HBM / MALL round trips per quad (5.6-11.6 us per call at
// c2's split 12 / 16, profiles/r03e_c2_by_kernel.txt).  KS = 0: any count, four loads
// in flight per trip.  One quad per thread (no grid-stride trips).
// S16: fp16 partials (IgemmParams::slab16), converted and summed in fp32.
template <bool S16>
__device__ __forceinline__ f32x4 slab_quad(const float* ws, size_t off) {
    if constexpr (S16) {
        const f16x4 h = *reinterpret_cast<const f16x4*>(reinterpret_cast<const f16*>(ws) + off);
        return (f32x4){(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    } else {
        return *reinterpret_cast<const f32x4*>(ws + off);
    }
}

template <int KS, bool S16>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(IgemmParams p) {
    const int cq = p.cout >> 2;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)p.M * cq) return;
    const int hw = p.oh * p.ow;
    const size_t slab = (size_t)p.M * p.cout;
    const int m = (int)(i / cq);
    const int j = (int)(i - (size_t)m * cq) * 4;
    const size_t src = (size_t)m * p.cout + j;
    float4 bv = {0.f, 0.f, 0.f, 0.f};
    f16x4 tv = {0, 0, 0, 0}, rv = {0, 0, 0, 0};
    if (p.bias) bv = *reinterpret_cast<const float4*>(p.bias + j);
    if (p.temb) tv = *reinterpret_cast<const f16x4*>(p.temb + (size_t)(m / hw) * p.temb_ld + j);
    if (p.resid) rv = *reinterpret_cast<const f16x4*>(p.resid + (size_t)m * p.resid_ld + j);
    f32x4 acc;
    if constexpr (KS > 0) {
        f32x4 v[KS];
#pragma unroll
        for (int sl = 0; sl < KS; ++sl) v[sl] = slab_quad<S16>(p.ws, src + sl * slab);
        acc = v[0];
#pragma unroll
        for (int sl = 1; sl < KS; ++sl) acc += v[sl];
    } else {
        acc = slab_quad<S16>(p.ws, src);
        int sl = 1;
        for (; sl + 4 <= p.ksplit; sl += 4) {
            const f32x4 a = slab_quad<S16>(p.ws, src + sl * slab);
            const f32x4 b = slab_quad<S16>(p.ws, src + (sl + 1) * slab);
            const f32x4 c = slab_quad<S16>(p.ws, src + (sl + 2) * slab);
            const f32x4 d = slab_quad<S16>(p.ws, src + (sl + 3) * slab);
            acc += a; acc += b; acc += c; acc += d;
        }
        for (; sl < p.ksplit; ++sl) acc += slab_quad<S16>(p.ws, src + sl * slab);
    }
    float v[4] = {acc[0] + bv.x, acc[1] + bv.y, acc[2] + bv.z, acc[3] + bv.w};
    f16x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        if (p.act == C2D_ACT_GELU) v[r] = gelu_f(v[r]);
        else if (p.act == C2D_ACT_RELU) v[r] = fmaxf(v[r], 0.f);
        else if (p.act == C2D_ACT_SILU) v[r] = silu_f(v[r]);
        else if (p.act == C2D_ACT_QUICK_GELU) v[r] = sigmoid_lin(v[r], 1.702f);
        if (p.temb) v[r] += (float)tv[r];
        if (p.resid) v[r] += (float)rv[r];
        o[r] = (f16)v[r];
    }
    *reinterpret_cast<f16x4*>(p.out + (size_t)m * p.out_ld + j) = o;
}

// Split-K combine that also emits the output's GroupNorm moments (IgemmParams::gn_mom): block = kGnRb rows x
// 320 columns of one image, 640 threads; thread t owns columns 4 (t % 80) .. +3 of rows t / 80 and t / 80 + 8,
// every slab load of both issued before the first add (as splitk_reduce_kernel's one quad per thread: the
// combine stays a single round of HBM / L2 latency).  Each output goes through splitk_reduce_kernel's
// arithmetic; the thread forms the exact (mean, M2) of its two fp16-rounded values per column, the eight
// row threads of a column merge in LDS (Chan, equal counts, fixed order), then each group's columns.
// Writes {mean, M2} per (image, kGnRb-row block, group): the layout c2d_groupnorm_moments reads.
constexpr int kGnRb = 16;
template <int KS, bool S16>
__global__ void __launch_bounds__(640) splitk_reduce_gn_kernel(IgemmParams p) {
    __shared__ float2 cm[8][320];
    const int t = threadIdx.x, q = t % 80, rs = t / 80;
    const int m0 = blockIdx.x * kGnRb, j = blockIdx.y * 320 + 4 * q;
    const int hw = p.oh * p.ow;
    const size_t slab = (size_t)p.M * p.cout;
    float4 bv = {0.f, 0.f, 0.f, 0.f};
    f16x4 tv = {0, 0, 0, 0}, rv[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
    if (p.bias) bv = *reinterpret_cast<const float4*>(p.bias + j);
    if (p.temb) tv = *reinterpret_cast<const f16x4*>(p.temb + (size_t)(m0 / hw) * p.temb_ld + j);
    f32x4 v[2][KS];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int m = m0 + rs + 8 * i;
        if (p.resid) rv[i] = *reinterpret_cast<const f16x4*>(p.resid + (size_t)m * p.resid_ld + j);
#pragma unroll
        for (int sl = 0; sl < KS; ++sl) v[i][sl] = slab_quad<S16>(p.ws, (size_t)m * p.cout + j + sl * slab);
    }
    float y[2][4];
    const float b4[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        f32x4 acc = v[i][0];
#pragma unroll
        for (int sl = 1; sl < KS; ++sl) acc += v[i][sl];
        f16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float x = acc[r] + b4[r];
            if (p.temb) x += (float)tv[r];
            if (p.resid) x += (float)rv[i][r];
            o[r] = (f16)x;
            y[i][r] = (float)o[r];
        }
        *reinterpret_cast<f16x4*>(p.out + (size_t)(m0 + rs + 8 * i) * p.out_ld + j) = o;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {   // two values: mean, M2 = (a - b)^2 / 2
        const float d = y[0][r] - y[1][r];
        cm[rs][4 * q + r] = make_float2(0.5f * (y[0][r] + y[1][r]), 0.5f * d * d);
    }
    __syncthreads();
    float2 col = {0.f, 0.f};
    if (t < 320) {   // per column t: merge the eight row threads (equal counts 2)
        float mu = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) mu += cm[k][t].x;
        mu *= 0.125f;
        float m2 = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float d = cm[k][t].x - mu;
            m2 += cm[k][t].y + 2.0f * d * d;
        }
        col = make_float2(mu, m2);
    }
    __syncthreads();
    if (t < 320) cm[0][t] = col;
    __syncthreads();
    const int cpg = p.gn_cpg, ng = 320 / cpg;
    if (t < ng) {   // per group: its columns (equal counts kGnRb)
        float mg = 0.f;
        for (int i = 0; i < cpg; ++i) mg += cm[0][t * cpg + i].x;
        mg /= (float)cpg;
        float m2 = 0.f;
        for (int i = 0; i < cpg; ++i) {
            const float d = cm[0][t * cpg + i].x - mg;
            m2 += cm[0][t * cpg + i].y + (float)kGnRb * d * d;
        }
        const int nimg = m0 / hw, groups = p.cout / cpg;
        const size_t slot = ((size_t)nimg * (hw / kGnRb) + (m0 - nimg * hw) / kGnRb) * groups + blockIdx.y * ng + t;
        reinterpret_cast<float2*>(p.gn_mom)[slot] = make_float2(mg, m2);
    }
}

void run_splitk_reduce(const IgemmParams& p, hipStream_t s) {
    if (p.gn_mom) {   // gn_rows_for: cout % 320 == 0, hw % kGnRb == 0, act none
        const dim3 grid((unsigned)(p.M / kGnRb), (unsigned)(p.cout / 320)), blk(640);
#define C2D_SKG(KS)                                                                                    \
    if (p.slab16) hipLaunchKernelGGL((splitk_reduce_gn_kernel<KS, true>), grid, blk, 0, s, p);        \
    else hipLaunchKernelGGL((splitk_reduce_gn_kernel<KS, false>), grid, blk, 0, s, p)
        switch (p.ksplit) {
            case 2: C2D_SKG(2); break;
            case 3: C2D_SKG(3); break;
            case 4: C2D_SKG(4); break;
            case 5: C2D_SKG(5); break;
            case 6: C2D_SKG(6); break;
            case 8: C2D_SKG(8); break;
            case 10: C2D_SKG(10); break;
            case 12: C2D_SKG(12); break;
            case 15: C2D_SKG(15); break;
            default: C2D_SKG(16); break;   // gn_split_ok: only the counts above and 16
        }
#undef C2D_SKG
        return;
    }
    const size_t total = (size_t)p.M * (p.cout >> 2);
    const dim3 grid((unsigned)((total + 255) / 256)), blk(256);
#define C2D_SKR(KS)                                                                   \
    if (p.slab16) hipLaunchKernelGGL((splitk_reduce_kernel<KS, true>), grid, blk, 0, s, p); \
    else hipLaunchKernelGGL((splitk_reduce_kernel<KS, false>), grid, blk, 0, s, p)
    switch (p.ksplit) {
        case 2: C2D_SKR(2); break;
        case 3: C2D_SKR(3); break;
        case 4: C2D_SKR(4); break;
        case 6: C2D_SKR(6); break;
        case 8: C2D_SKR(8); break;
        case 12: C2D_SKR(12); break;
        case 16: C2D_SKR(16); break;
        default: C2D_SKR(0); break;
    }
#undef C2D_SKR
}
#else
void run_splitk_reduce(const IgemmParams& p, hipStream_t s);
#endif

}  // namespace c2d
#include "igemm_m32.h"
#include "igemm_pp16.h"
#include "igemm_pps.h"
#include "igemm_pp16r.h"
#include "igemm_panel.h"
namespace c2d {

template <int WM, int WN, int TM, int TN, int STAGES, int KS, int KG = 1>
static void launch_dma(const IgemmParams& p, hipStream_t s) {
    // the KG rings, or the fp32 epilogue image (per wave 16 * min(TM, 2) rows x (TN * 16 + 4)
    // floats) that reuses them after the main loop (KG > 1: plus the other groups' accumulators
    // above it), whichever is larger
    constexpr int ring = KG * STAGES * (WM * TM + WN * TN) * 16 * 128;
    constexpr int epi0 = WM * WN * 16 * (TM < 2 ? TM : 2) * (TN * 16 + 4) * 4;
    constexpr int epi = KG > 1 ? (epi0 + 1023) / 1024 * 1024 + (KG - 1) * WM * WN * TM * TN * 1024 : epi0;
    constexpr int smem = ring > epi ? ring : epi;
    static_assert(smem <= 160 * 1024, "LDS ring / epilogue image too large");
    auto k = igemm_dma_kernel<WM, WN, TM, TN, STAGES, KS, KG>;
    ensure_lds<igemm_dma_kernel<WM, WN, TM, TN, STAGES, KS, KG>>(smem);
    hipLaunchKernelGGL(k, dim3(p.gx * p.gy * p.ksplit), dim3(64 * WM * WN * KG), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

template <int BM, int BN, int AMODE>
static void launch(const IgemmParams& p, hipStream_t s) {
    const int smem = 2 * (BM + BN) * 128;
    dim3 grid(p.gx * p.gy);
    hipLaunchKernelGGL((igemm_kernel<BM, BN, AMODE>), grid, dim3(256), smem, s, p);
}

}  // namespace c2d

using namespace c2d;

// C2D_TUNE_GEMM_MODE=2 (variant build) restricts to the register-staged kernels (A/B
// comparisons, debugging); default 0 = auto.
static int gemm_mode() { return tuning().gemm_mode; }

// c2d_set_plan_override(tile, split): force DMA tile config `tile` (shape sweeps, the
// per-tile parity test); 0 = heuristic.  An explicit setter, never the environment.
static int gemm_tile() { return plan_override_tile(); }

template <int WM, int WN, int TM, int TN, int ST, int KG = 1>
static void run_dma(IgemmParams& p, int ksize, int cout, hipStream_t s) {
    constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
    p.gx = (cout + BN - 1) / BN;
    p.gy = (p.M + BM - 1) / BM;
    if (ksize == 1) launch_dma<WM, WN, TM, TN, ST, 1, KG>(p, s);
    else launch_dma<WM, WN, TM, TN, ST, 3, KG>(p, s);
}

// One wrapper per DMA tile id, each compiled in its kernel family's part.
#define C2D_TILE_FN(ID) void run_tile_##ID(IgemmParams& p, int ksize, int cout, hipStream_t s)
namespace c2d {
C2D_TILE_FN(25); C2D_TILE_FN(40); C2D_TILE_FN(41); C2D_TILE_FN(28); C2D_TILE_FN(29);
C2D_TILE_FN(7); C2D_TILE_FN(1); C2D_TILE_FN(2); C2D_TILE_FN(3); C2D_TILE_FN(50); C2D_TILE_FN(8); C2D_TILE_FN(9);
C2D_TILE_FN(42); C2D_TILE_FN(43); C2D_TILE_FN(44); C2D_TILE_FN(70); C2D_TILE_FN(80); C2D_TILE_FN(81);
#if C2D_PART(1)
C2D_TILE_FN(40) { run_pp16<5>(p, ksize, cout, s); }   // 256x320 ping-pong 16x16x32
C2D_TILE_FN(41) { run_pp16<4>(p, ksize, cout, s); }   // 256x256 ping-pong 16x16x32
C2D_TILE_FN(50) { (void)ksize; (void)cout; run_pps(p, s); }   // persistent 192x256, carried epilogue (1x1)
C2D_TILE_FN(42) { (void)ksize; (void)cout; run_pp16r<5>(p, 42, s); }   // 256x320 row-ring 3x3, output width 64
C2D_TILE_FN(43) { (void)ksize; (void)cout; run_pp16r<5>(p, 43, s); }   // 128x320 row-ring 3x3, output width 32
C2D_TILE_FN(44) { (void)ksize; (void)cout; run_pp16r<5>(p, 44, s); }   // 128x320 row-ring 3x3, output width 16
#endif
#if C2D_PART(2)
C2D_TILE_FN(25) { run_m32<4, 2, 2, 5, 64, 2, 3, 0, true>(p, ksize, cout, s); }   // 256x320, 8 waves of 64x160
C2D_TILE_FN(28) { run_m32<4, 2, 2, 4, 64, 2, 3>(p, ksize, cout, s); }            // 256x256, 8 waves of 64x128
C2D_TILE_FN(29) { run_m32<4, 2, 2, 2, 64, 3, 3>(p, ksize, cout, s); }            // 256x128, 8 waves of 64x64, 3 stages
#endif
#if C2D_PART(3)
C2D_TILE_FN(7) { run_dma<2, 4, 4, 5, 2>(p, ksize, cout, s); }   // 128x320, 8 waves of 64x80
C2D_TILE_FN(1) { run_dma<4, 2, 4, 4, 3>(p, ksize, cout, s); }   // 256x128, 8 waves of 64x64
C2D_TILE_FN(2) { run_dma<2, 2, 4, 4, 3>(p, ksize, cout, s); }   // 128x128, 4 waves of 64x64
C2D_TILE_FN(3) { run_dma<2, 2, 2, 2, 3>(p, ksize, cout, s); }   // 64x64, 4 waves of 32x32
C2D_TILE_FN(8) { run_dma<2, 2, 4, 5, 2>(p, ksize, cout, s); }   // 128x160, 4 waves of 64x80, 72 KiB: 2 per CU
C2D_TILE_FN(9) { run_dma<2, 2, 2, 5, 2>(p, ksize, cout, s); }   // 64x160, 4 waves of 32x80, 56 KiB: 2 per CU
C2D_TILE_FN(80) { run_dma<2, 2, 4, 5, 2, 2>(p, ksize, cout, s); }   // 128x160, 2 K groups of 4 waves of 64x80, 144 KiB
C2D_TILE_FN(81) { run_dma<2, 2, 2, 5, 2, 2>(p, ksize, cout, s); }   // 64x160, 2 K groups of 4 waves of 32x80, 112 KiB
#endif
#if C2D_PART(4)
C2D_TILE_FN(70) { (void)ksize; (void)cout; run_panel(p, s); }   // 128-row A panel in LDS, weights streamed per wave
#endif
}  // namespace c2d
#undef C2D_TILE_FN

#if C2D_PART(0)
// Tile / split-K choice from a cost model: estimated time = rounds of resident
// blocks x per-block time (K steps + a fill/epilogue overhead, at the per-CU
// rate measured on gfx950 for that tile with the CU full) + the split-K combine
// (fp32 slabs written and read once, HBM rate, one extra launch).  The 128x320
// tile fits SD's channel counts (all multiples of 320) with no column waste but
// has an odd per-wave column-tile count, so GEGLU skips it; GEGLU never splits.
struct DmaTile { int id, bm, bn, occ; float rate; bool geglu; };
static const DmaTile kDmaTiles[] = {
    // 32x32x16 MFMA, LDS-DMA ring (igemm_m32.h); rate 0 = chosen by the rules in plan_for only
    {25, 256, 320, 1, 0.0f, true},
    {40, 256, 320, 1, 0.0f, false},   // ping-pong 16x16x32 (80-column wave tiles: no GEGLU pairs in the plain epilogue)
    {41, 256, 256, 1, 0.0f, true},
    {28, 256, 256, 1, 0.0f, true},
    {29, 256, 128, 1, 0.0f, true},
    // 16x16x32 MFMA LDS-DMA family, costed by plan_dma
    {7, 128, 320, 1, 3.1f, false},
    {1, 256, 128, 1, 2.9f, true},
    {2, 128, 128, 1, 2.2f, true},
    {3, 64, 64, 3, 1.9f, true},
    // two workgroups per CU (<= 80 KiB of LDS): the under-filled 1x1 / 3x3 shapes
    {8, 128, 160, 2, 0.0f, false},
    {9, 64, 160, 2, 0.0f, false},
    // tiles 8 / 9 with two K groups in one workgroup (intra-workgroup split-K, 8 waves, one per CU)
    {80, 128, 160, 1, 0.0f, false},
    {81, 64, 160, 1, 0.0f, false},
    // row-ring 3x3 over a zero-bordered source (igemm_pp16r.h), one per output width (64 / 32 / 16):
    // chosen by plan_for only
    {42, 256, 320, 1, 0.0f, false},
    {43, 128, 320, 1, 0.0f, false},
    {44, 128, 320, 1, 0.0f, false},
};
struct DmaPlan { int id, split, nkt; };

static DmaPlan plan_dma(long M, int cout, int nk, bool geglu, int force_id, int force_split) {
    DmaPlan best = {3, 1, nk};
    double best_t = 1e300;
    // 12 / 16 only by a forced plan or the measured table (the cost model is not calibrated there)
    const int splits[] = {1, 2, 3, 4, 6, 8, 12, 16};
    for (const DmaTile& t : kDmaTiles) {
        if (geglu && !t.geglu) continue;
        if (force_id && t.id != force_id) continue;
        if (!force_id && t.rate <= 0.f) continue;
        const long tiles = ((M + t.bm - 1) / t.bm) * ((cout + t.bn - 1) / t.bn);
        for (int sp : splits) {
            if (force_split && sp != force_split) continue;
            if (!force_split && sp > 8) continue;
            if (sp > 1 && (geglu || nk < 8 * sp || tiles >= 256)) continue;
            const int nkt = (nk + sp - 1) / sp;
            const int eff = (nk + nkt - 1) / nkt;
            const long blocks = tiles * eff;
            const long slots = 256L * t.occ;
            const double blk_us = 2.0 * t.bm * t.bn * 64.0 * (nkt + 3) * t.occ / ((t.rate > 0.f ? t.rate : 3.0f) * 1e6);
            double est = (double)((blocks + slots - 1) / slots) * blk_us;
            if (eff > 1) est += (double)M * cout * 4.0 * (eff + 1) / 4e6 + 2.0;
            if (est < best_t) { best_t = est; best = {t.id, eff, nkt}; }
        }
    }
    return best;
}

// C2D_GEMM_ABL: timing ablation of the DMA kernels (1 = no DMA, 2 = no MFMA; m32: 4 = no epilogue,
// 8 = with 2, no fragment reads either); wrong results by design, so only in -DC2D_ENABLE_ABLATION builds
static int gemm_abl() { return ablation_gemm(); }

// K-step order of the 3x3 DMA kernels.  1 (default): for each 64-channel block all
// 9 taps, so one block re-reads a (rows + 2 halo image rows) x 64-channel slab from
// L2 nine times in a row (~1.6 MB live per XCD at 32 resident 256-row blocks).
// 0: tap-major, the packed weight order, whose reuse distance (rows x cin) spills
// the 4 MB L2 at cin = 320 and re-fetches the input over the fabric once per tap.
static int gemm_korder() { return tuning().gemm_korder; }

// C2D_TUNE_GEMM_LDSEPI=0 (variant build) lets the 32x32 GEGLU GEMMs store straight from the accumulators:
// 10 % faster in isolation (L0 320 -> 2 x 1280) but 0.3 % slower in the full step
// (same-box bench A/B, twice each), so the LDS-staged epilogue stays the default
static int gemm_lds_epi() { return tuning().gemm_lds_epi; }

// the direct 32x32 epilogue stores 4-channel (8-B) runs and loads the bias as float4
static bool epi_direct_ok(const c2d_conv_desc* d) {
    const int out_cols = d->act == C2D_ACT_GEGLU ? d->cout / 2 : d->cout;
    const uintptr_t a8 = (uintptr_t)d->out | (uintptr_t)d->resid | (uintptr_t)d->temb;
    return (out_cols % 4) == 0 && (d->out_ld % 4) == 0 && (!d->resid || (d->resid_ld % 4) == 0) &&
           (!d->temb || (d->temb_ld % 4) == 0) && (a8 & 7) == 0 && ((uintptr_t)d->bias & 15) == 0;
}

// c2d_set_plan_override's split (when the workspace allows); 0 = model
static int gemm_split() { return plan_override_split(); }

// Tile choice.  Measured on gfx950 over the UNet's conv / linear shapes
// (scripts/bench_gemm.py, scripts/sweep_tiles_graph.py): the 256x320 32x32-MFMA tile
// (id 23) is fastest whenever its tiles fill the chip by themselves (all level-0
// GEMMs, the GEGLU projections, the 256-row-tile-rich up-block convs); otherwise
// the 128x320 tile (id 7; GEGLU: 256x128, id 1) when its tiles fill the chip;
// under-filled shapes (16x16 / 8x8 levels) go through the cost model with split-K.
// the persistent carried-epilogue kernel (tile 50, igemm_pps.h): 1x1, plain output (no
// residual / time embedding, act none or GEGLU), K = 320 / 640 / 1280, 8-B aligned output,
// 32-bit buffer offsets
static bool pps_eligible(const c2d_conv_desc* d) {
    const long M = (long)d->n * d->oh * d->ow;
    return d->ksize == 1 && !d->resid && !d->temb && (d->act == C2D_ACT_NONE || d->act == C2D_ACT_GEGLU) &&
           pps_nk_ok(d->kpad / 64) && (d->out_ld % 4) == 0 && ((uintptr_t)d->out & 7) == 0 &&
           ((uintptr_t)d->bias & 15) == 0 && (size_t)M * d->out_ld * 2 < (1u << 31);
}

// Measured plans for the SD1.5 UNet shapes where the rules below lose >= 3 %: graph-replayed
// forced-(tile, split) sweeps on MI355X at the three batches the configurations run
// (scripts/sweep_tiles_graph.py; profiles/r03_sweep_b1.txt, r03_sweep_b4r96.txt,
// r03_sweep_b8.txt; r03_sweep2.txt: split-K 12 / 16 for the N = 2 small-M convs;
// r03_sweep_fold.txt: the K = 5C ff.net.2 + proj_out GEMMs).  The rules
// are tuned on N = 16 at 64^2; at N = 2 (c1 / c2) every shape is latency bound, and at 96^2
// (c5) the 256-row tile count is 288 = 1.1 rounds of 256 CUs.
// Keyed on (ksize, M = N * H * W, kpad, cout, GEGLU); anything else goes through the rules.
struct PlanHint { int ksize; long M; int kpad, cout; bool geglu; int id, split; };
static const PlanHint kPlanHints[] = {
    // N = 2, 64^2 (c1 / c2 latency)
    {1, 8192, 1280, 320, false, 9, 1},        // ff2 L0: 18.5 -> 17.4 us
    {1, 2048, 640, 1920, false, 9, 1},        // QKV L1: 13.7 -> 13.0
    {1, 512, 1280, 1280, false, 3, 1},        // 1x1 L2: 14.0 -> 10.8
    {1, 2048, 640, 5120, true, 50, 1},        // GEGLU L1: 32.7 -> 24.9 (persistent, 220 tiles)
    {3, 8192, 2880, 320, false, 7, 4},        // 3x3 L0 320: 49.3 -> 39.7
    {3, 8192, 5760, 320, false, 40, 6},       // 3x3 L0 640 -> 320: 58.2 -> 54.7
    {3, 8192, 8640, 320, false, 40, 8},       // 3x3 L0 960 -> 320: 72.8 -> 66.9
    {3, 2048, 5760, 640, false, 7, 8},        // 3x3 L1 640: 42.3 -> 38.7
    {3, 2048, 17280, 640, false, 40, 16},     // 3x3 L1 1920 -> 640: 73.4 -> 67.0 (r04 fp32 slabs)
    {3, 512, 11520, 1280, false, 7, 12},      // 3x3 L2 1280: 55.2 -> 43.7 (split 12)
    {3, 512, 17280, 1280, false, 41, 16},     // 3x3 L2 1920 -> 1280: 75.2 -> 48.3
    {3, 512, 23040, 1280, false, 41, 16},     // 3x3 L2 2560 -> 1280: 95.4 -> 57.1
    {3, 128, 11520, 1280, false, 81, 12},     // 3x3 L3 1280: 31.4 -> 25.7 (3, 12); r06 two K groups (81, 12): 23.8 -> 22.0
    {3, 128, 23040, 1280, false, 81, 12},     // 3x3 L3 2560 -> 1280: 52.6 -> 38.1 (9, 16); r06 (81, 12): 36.4 -> 32.3
    {1, 2048, 3200, 640, false, 81, 2},       // ff.net.2 + proj_out fold L1 (K = 5C): r06 (2, 3) 24.6 -> (81, 2) 22.9
    {1, 128, 6400, 1280, false, 3, 12},       // ff.net.2 + proj_out fold L3 (K = 5C): 15.0 -> 14.4
    // N = 8, 96^2 (c5)
    {1, 73728, 320, 320, false, 7, 1},        // 1x1 L0: 53.9 -> 41.6
    {1, 73728, 1280, 320, false, 7, 1},       // ff2 L0: 120.7 -> 104.6
    {1, 18432, 640, 640, false, 41, 1},       // 1x1 L1: 38.2 -> 31.9
    {1, 18432, 2560, 640, false, 41, 1},      // ff2 L1: 101.2 -> 74.6
    {1, 4608, 5120, 1280, false, 40, 3},      // ff2 L2: 83.2 -> 79.2
    {1, 4608, 1280, 10240, true, 41, 1},      // GEGLU L2: 153.8 -> 138.5
    {1, 1152, 1280, 1280, false, 3, 1},       // 1x1 L3: 18.5 -> 15.6
    {3, 18432, 5760, 640, false, 41, 1},      // 3x3 L1 640: 163.0 -> 147.7
    {3, 1152, 11520, 1280, false, 41, 8},     // 3x3 L3 1280: 65.4 -> 61.2
    {3, 1152, 23040, 1280, false, 41, 8},     // 3x3 L3 2560 -> 1280: 116.7 -> 96.1
    {1, 1152, 6400, 1280, false, 80, 3},      // ff.net.2 + proj_out fold L3: r06 (7, 6) 41.6 -> (80, 3) 39.5
    {1, 73728, 1600, 320, false, 7, 1},       // ff.net.2 + proj_out fold L0: 145.6 -> 136.9
    {1, 18432, 3200, 640, false, 41, 1},      // fold L1: 121.9 -> 87.7
    // the panel GEMM (tile 70, igemm_panel.h), graph-replayed forced sweeps at the three batches
    // (profiles/r05_panel_gemm.txt); -DC2D_NO_PANEL_HINTS: A/B builds without them
#ifndef C2D_NO_PANEL_HINTS
    {1, 65536, 320, 2560, true, 70, 1},       // c3 GEGLU L0: 154.7 -> 120.4 us
    {1, 16384, 640, 5120, true, 70, 1},       // c3 GEGLU L1: 135.0 -> 117.7
    {1, 65536, 320, 960, false, 70, 1},       // c3 QKV L0: 68.8 -> 65.2
    {1, 73728, 320, 2560, true, 70, 1},       // c5 GEGLU L0: 173.8 -> 157.7
    {1, 8192, 320, 2560, true, 70, 1},        // c2 GEGLU L0: 25.9 -> 20.7
    {1, 8192, 320, 960, false, 70, 1},        // c2 QKV L0: 13.9 -> 12.5
#endif
    // N = 16, 64^2 (c3)
    {1, 4096, 1280, 1280, false, 80, 1},      // 1x1 L2: 27.2 -> 24.5 (8, 1); r06 two K groups (80, 1): +res 26.0 -> 24.9, plain 24.7 -> 22.9
    {1, 1024, 1280, 1280, false, 3, 1},       // 1x1 mid: 18.9 -> 13.5
    {3, 1024, 11520, 1280, false, 41, 12},    // 3x3 L3 1280: 61.2 -> 52.5 (r04 re-sweep, fp32 slabs)
    {3, 1024, 23040, 1280, false, 41, 12},    // 3x3 L3 2560 -> 1280: 97.2 -> 91.3 (split 8); 87.9 -> 77.3 (r04: 12)
    {1, 4096, 6400, 1280, false, 80, 1},      // ff.net.2 + proj_out fold L2: 84.7 -> 82.2 (7, 2); r06 (80, 1): 82.2 -> 76.1
    // VAE decoder at batch 8 (profiles/r03_sweep_vae.txt): only the 1x1 shortcuts gain
    {1, 2097152, 256, 128, false, 1, 1},      // 512^2 256 -> 128: 511.9 -> 459.4
    {1, 524288, 512, 256, false, 1, 1},       // 256^2 512 -> 256: 307.5 -> 294.3
};

static bool plan_hint(int ksize, long M, int kpad, int cout, bool geglu, DmaPlan& pl) {
    for (const PlanHint& h : kPlanHints)
        if (h.ksize == ksize && h.M == M && h.kpad == kpad && h.cout == cout && h.geglu == geglu) {
            const int nk = kpad / 64;
            const int nkt = (nk + h.split - 1) / h.split;
            pl = {h.id, (nk + nkt - 1) / nkt, nkt};
            return true;
        }
    return false;
}

// Measured row-ring plans (tile, split) for zero-bordered-source 3x3 shapes where the rules below
// lose >= 3 % to one (scripts/rr_sweep.py: the production route on the unpadded source against the
// row-ring tile with every split of whole channel blocks, graph-replayed, profiles/r06_rr_sweep_*.txt).
// Keyed on (M = N * H * W, kpad, cout); only consulted when the descriptor's width has a row-ring tile.
struct RrHint { long M; int kpad, cout, id, split; };
static const RrHint kRrHints[] = {
    // N = 2 (c1 / c2; profiles/r06_rr_sweep_b1.txt): every ResnetBlock2D 3x3 of levels 0-2 except the
    // level-0 320 -> 320 (tied with (7, 4) on the unpadded source)
    {8192, 5760, 320, 42, 5},   // N = 2 64^2 640 -> 320: 56.7 -> 51.9 us
    {8192, 8640, 320, 42, 8},   // N = 2 64^2 960 -> 320: 71.2 -> 63.1 us
    {2048, 2880, 640, 43, 5},   // N = 2 32^2 320 -> 640: 34.5 -> 26.2 us
    {2048, 5760, 640, 43, 5},   // N = 2 32^2 640 -> 640: 40.1 -> 33.6 us
    {2048, 8640, 640, 43, 8},   // N = 2 32^2 960 -> 640: 49.3 -> 39.7 us
    {2048, 11520, 640, 43, 5},   // N = 2 32^2 1280 -> 640: 59.8 -> 49.3 us
    {2048, 17280, 640, 43, 8},   // N = 2 32^2 1920 -> 640: 73.6 -> 58.6 us
    {512, 5760, 1280, 44, 10},   // N = 2 16^2 640 -> 1280: 34.7 -> 27.8 us
    {512, 11520, 1280, 44, 10},   // N = 2 16^2 1280 -> 1280: 44.2 -> 36.2 us
    {512, 17280, 1280, 44, 15},   // N = 2 16^2 1920 -> 1280: 50.1 -> 45.3 us
    {512, 23040, 1280, 44, 10},   // N = 2 16^2 2560 -> 1280: 59.8 -> 53.6 us
};

// a row-ring tile of the same geometry as rr_id (one tile per width today)
static bool rr_compatible(int id, int rr_id) { return id == rr_id; }

static bool rr_hint(long M, int kpad, int cout, int rr_id, int& id, int& split) {
    for (const RrHint& h : kRrHints)
        if (h.M == M && h.kpad == kpad && h.cout == cout && rr_compatible(h.id, rr_id)) {
            id = h.id;
            split = h.split;
            return true;
        }
    return false;
}

// row-ring plan (tiles 42 / 43 / 44): split-K slices own whole channel blocks (9 K steps each)
static DmaPlan rr_plan(int id, int nk, int split) {
    const int ncb = nk / 9;
    const int sp = split < 1 ? 1 : (split > ncb ? ncb : split);
    const int cbs = (ncb + sp - 1) / sp;
    return {id, (ncb + cbs - 1) / cbs, 9 * cbs};
}

// rr_id: the row-ring tile this descriptor can run on (rr_tile), 0 = none
static DmaPlan plan_for(long M, int cout, int kpad, int act, bool pps_ok, int ksize, int rr_id = 0,
                        bool panel_ok = false) {
    const bool geglu = act == C2D_ACT_GEGLU;
    const int nk = kpad / 64;
    int id = gemm_tile();
    if (id == 70) {   // the panel GEMM (igemm_panel.h): one slice, no split
        if (panel_ok && gemm_split() <= 1) return {70, 1, nk};
        id = 0;
    }
    if (id == 42 || id == 43 || id == 44) {
        if (rr_id && rr_compatible(id, rr_id)) return rr_plan(id, nk, gemm_split());
        id = 0;
    }
    // the row-ring 3x3 on a zero-bordered source once its tiles fill the chip: tile 42 (256 x 320,
    // width 64: c3's level-0 ResnetBlock2D convs), tile 43 (128 x 320, width 32: level 1, 256 tiles
    // at N = 16 with no split), tile 44 (128 x 320, width 16: level 2, 128 tiles -> 2 K slices);
    // under-filled grids keep the planner's tiles over the padded image (a valid 3x3, every tap in
    // bounds).  Graph-replayed per-shape A/B (scripts/rowring_ab.py, profiles/r06_rowring_ab.txt):
    // tile 43 beats (40, 2) by 5-11 % up to 15 channel blocks (640 +res 125.3 -> 111.6 us) and loses
    // 2 % at 30 (the 1920 -> 640 up-block conv, whose 270 K steps amortise the split's combine);
    // tile 44 (2 slices) beats (40, 4) at 10 channel blocks, ties at 20, loses at 40
    if (!id && rr_id && !gemm_split()) {
        int hid = 0, sp = 0;
        if (rr_hint(M, kpad, cout, rr_id, hid, sp)) return rr_plan(hid, nk, sp);
    }
    if (!id && rr_id && !gemm_split() && cout % 320 == 0) {
        const long tiles = (M / (rr_id == 42 ? 256 : 128)) * (cout / 320);
        const int ncb = nk / 9;
        if (tiles >= 192 && (rr_id != 43 || ncb < 30)) return rr_plan(rr_id, nk, 1);
        if (rr_id == 44 && tiles >= 96 && ncb >= 4 && ncb <= 10) return rr_plan(rr_id, nk, 2);
    }
    if (!id && !gemm_split()) {   // a forced split (tile left to the planner) skips the table
        DmaPlan pl;
        if (plan_hint(ksize, M, kpad, cout, geglu, pl) && (pl.id != 50 || pps_ok) && (pl.id != 70 || panel_ok)) return pl;
    }
    if (id == 7 && geglu) id = 0;
    if (id == 50) {
        if (pps_ok) return {50, 1, nk};
        id = 0;
    }
    // GEGLU with K = 320 / 640 on the chip-filling grids: the persistent carried-epilogue
    // kernel (same box, scripts/ab_tiles.py: L0 320 -> 2 x 1280 187 -> 166 us, L1 640 -> 2 x 2560
    // 147 -> 138 us; K = 1280 and the plain outputs stay on the one-shot tiles, where its
    // 192 x 256 tile's extra DMA per MAC costs more than the overlap saves)
    if (!id && pps_ok && geglu && (nk == 5 || nk == 10) && ((M + 191) / 192) * ((cout + 255) / 256) >= 512)
        return {50, 1, nk};
    if (id) {
        DmaPlan pl = plan_dma(M, cout, nk, geglu, id, gemm_split());
        if (pl.id) return pl;
    }
    // narrow outputs (the UNet / VAE conv_out, 4 channels): the 256x128 32x32-MFMA tile, 3
    // stages (scripts/small_cout.py, forced tiles on one box: UNet conv_out 320 -> 4 at 64^2,
    // N = 16: 91.3 us on tile 40, 80.5 on the 64x64 tile 3, 49.0 on tile 29; VAE conv_out
    // 128 -> 4 at 512^2, N = 8: 1332.6 / 874.3 / 725.3 us)
    if (cout <= 64 && !geglu) {
        DmaPlan pl = plan_dma(M, cout, nk, geglu, 29, 0);
        if (pl.id == 29) return pl;
    }
    // rules from the shape sweeps (scripts/sweep_tiles_graph.py): the 256x320 interleaved-DMA
    // tile once it (nearly) fills the chip, and with split-K for the long-K convs
    // (9 * cin >= 5760: L1 / L2 resnet and up-block convs); 128x320 below that
    // VAE widths (128 / 256 / 512 channels) leave 320-wide tiles 20-60 % empty: the
    // 256x256 / 256x128 variants of the same kernel (512^2 x 128 ch conv: 250 vs 402 us;
    // 256 / 512 ch: 11-14 % faster)
    if (!geglu && cout % 320 != 0) {
        const long mt = (M + 255) / 256;
        if (C2D_PP16_DEFAULT && cout % 256 == 0 && mt * (cout / 256) >= 192) return {41, 1, nk};   // ping-pong 256x256 (VAE 256/512 ch)
        if (cout % 256 != 0 && cout % 128 == 0 && mt * (cout / 128) >= 192) return {29, 1, nk};
    }
    // 256x320: the ping-pong 16x16x32 kernel (tile 40, 5-12 % faster than the 32x32x16
    // tile 25 on every conv / K >= 320 GEMM shape measured, scripts/ab_tiles.py) except
    // for GEGLU, whose [16 h | 16 g] column pairs need 32-aligned per-wave column tiles in
    // the plain (per-wave image) epilogue
    const int t256x320 = (geglu || !C2D_PP16_DEFAULT) ? 25 : 40;
    const long t24 = ((M + 255) / 256) * ((cout + 319) / 320);
    if (t24 >= 192) {
        // 256 x 256 (tile 41) where its round count x tile width is smaller: the partial last
        // round of the 320-wide tiles costs a whole round (scripts/ab_tiles.py, same box:
        // L1 QKV 640 -> 1920 64.8 -> 57.8 us, L2 QKV 1280 -> 3840 54.0 -> 48.0 us; L0 QKV and
        // every 320 / 640-wide conv keep tile 40 by the same count)
        if (!geglu && C2D_PP16_DEFAULT) {
            const long mt = (M + 255) / 256;
            const long r40 = (t24 + 255) / 256, r41 = (mt * ((cout + 255) / 256) + 255) / 256;
            if (r41 * 256 < r40 * 320) return {41, 1, nk};
        }
        return {t256x320, 1, nk};
    }
    if (nk >= 90 && t24 >= 64) {
        DmaPlan pl = plan_dma(M, cout, nk, geglu, 25, 0);
        if (pl.id == 25) pl.id = t256x320;
        return pl;
    }
    const long t7 = geglu ? ((M + 255) / 256) * ((cout + 127) / 128) : ((M + 127) / 128) * ((cout + 319) / 320);
    if (t7 >= 256) return {geglu ? 1 : 7, 1, nk};
    return plan_dma(M, cout, nk, geglu, 0, 0);
}

static void dispatch_dma(IgemmParams& p, const DmaPlan& pl, int ksize, int cout, hipStream_t s) {
    p.ksplit = pl.split;
    p.nkt = pl.nkt;
    switch (pl.id) {
        case 42: return run_tile_42(p, ksize, cout, s);
        case 43: return run_tile_43(p, ksize, cout, s);
        case 44: return run_tile_44(p, ksize, cout, s);
        case 25: return run_tile_25(p, ksize, cout, s);
        case 40: return run_tile_40(p, ksize, cout, s);
        case 41: return run_tile_41(p, ksize, cout, s);
        case 28: return run_tile_28(p, ksize, cout, s);
        case 29: return run_tile_29(p, ksize, cout, s);
        case 50: return run_tile_50(p, ksize, cout, s);
        case 7: return run_tile_7(p, ksize, cout, s);
        case 1: return run_tile_1(p, ksize, cout, s);
        case 2: return run_tile_2(p, ksize, cout, s);
        case 8: return run_tile_8(p, ksize, cout, s);
        case 9: return run_tile_9(p, ksize, cout, s);
        case 80: return run_tile_80(p, ksize, cout, s);
        case 81: return run_tile_81(p, ksize, cout, s);
        case 70: return run_tile_70(p, ksize, cout, s);
        default: return run_tile_3(p, ksize, cout, s);
    }
}

// does this descriptor run on the LDS-DMA kernels (no prologue, buffer-offset limits)?
static bool dma_eligible(const c2d_conv_desc* d) {
    const int cin = d->c0 + d->c1;
    const int amode = (d->ksize == 1) ? AM_1X1 : ((cin % 64) == 0 ? AM_3X3_FAST : AM_3X3_GEN);
    const int pd = d->src_pad ? 2 : 0;
    const size_t src_bytes = (size_t)d->n * (d->h + pd) * (d->w + pd) * (size_t)(d->c0 > d->c1 ? d->c0 : d->c1) * 2;
    return (d->pro == C2D_PRO_NONE || d->pro == C2D_PRO_LNFOLD) && amode != AM_3X3_GEN && !d->up && gemm_mode() != 2 &&
           (d->c1 == 0 || (d->c0 & 63) == 0) && src_bytes < (1u << 31) &&
           (size_t)d->cout * d->kpad * 2 < (1u << 31);  // 32-bit buffer offsets
}

// the panel GEMM (tile 70, igemm_panel.h): 1x1, one source of 320 / 640 channels, K unpadded,
// 32-column blocks, no prologue / time embedding, act none or GEGLU (no residual), the direct
// epilogue's alignment
static bool panel_eligible(const c2d_conv_desc* d) {
    return d->ksize == 1 && d->c1 == 0 && (d->c0 == 320 || d->c0 == 640) && d->kpad == d->c0 && (d->cout & 31) == 0 &&
           (d->pro == C2D_PRO_NONE || (d->pro == C2D_PRO_LNFOLD && !d->resid)) &&
           !d->temb && (d->act == C2D_ACT_NONE || (d->act == C2D_ACT_GEGLU && !d->resid)) &&
           epi_direct_ok(d) && dma_eligible(d) && (size_t)d->n * d->oh * d->ow * d->out_ld * 2 < (1u << 31);
}

// the row-ring tile (igemm_pp16r.h: 42 / 43 / 44 by output width) this descriptor can run on, 0 = none
static int rr_eligible(const c2d_conv_desc* d) {
    if (!(d->src_pad && d->pro == C2D_PRO_NONE && d->oh == d->h && d->ow == d->w && d->kpad == 9 * d->c0)) return 0;
    return pp16r_tile_for(d->ksize, d->stride, 0, d->c1, d->c0, d->ow, d->oh, d->w + 2);
}

// Image split of a quantisation tail.  A one-slice plan whose grid is whole rounds of the chip plus
// at most a quarter round (c5's level-0 3x3 convs: 288 tiles of 256 x 320 on 256 CUs = one round
// + 32 tiles, the second round 1/8 full) runs as two launches: the first n1 images, whose tiles fit
// the whole rounds, on the plan; the rest on their own plan (split K over the idle CUs).  Only for
// deep K (>= 16 steps, so the extra launch is small against a round) and the planner's own choice
// (no override); returns n1, 0 = no split.
static int tail_images(const c2d_conv_desc* d, const DmaPlan& pl) {
    if (pl.split != 1 || d->n < 2 || d->pro != C2D_PRO_NONE || d->kpad / 64 < 16) return 0;
    if (plan_override_tile() || plan_override_split() || !tuning().tail_split) return 0;
    const DmaTile* t = nullptr;
    for (const DmaTile& x : kDmaTiles)
        if (x.id == pl.id) t = &x;
    if (!t) return 0;   // the persistent tile (50) walks its own grid
    const long hw = (long)d->oh * d->ow, slots = 256L * t->occ;
    const long gx = (d->cout + t->bn - 1) / t->bn;
    const long tiles = (d->n * hw + t->bm - 1) / t->bm * gx;
    const long full = tiles / slots * slots, rem = tiles - full;
    if (full == 0 || rem == 0 || rem > slots / 4) return 0;
    int n1 = d->n - 1;
    while (n1 > 0 && (n1 * hw + t->bm - 1) / t->bm * gx > full) --n1;
    return n1;
}

// the descriptor of images [n1, n): every per-image pointer advanced by n1 images
static c2d_conv_desc tail_desc(const c2d_conv_desc* d, int n1) {
    c2d_conv_desc t = *d;
    const size_t in_pix = (size_t)n1 * (d->src_pad ? (size_t)(d->h + 2) * (d->w + 2) : (size_t)d->h * d->w);
    const size_t out_rows = (size_t)n1 * d->oh * d->ow;
    t.n = d->n - n1;
    t.src0 = static_cast<const f16*>(d->src0) + in_pix * d->c0;
    if (d->src1) t.src1 = static_cast<const f16*>(d->src1) + in_pix * d->c1;
    if (d->temb) t.temb = static_cast<const f16*>(d->temb) + (size_t)n1 * d->temb_ld;
    if (d->resid) t.resid = static_cast<const f16*>(d->resid) + out_rows * d->resid_ld;
    t.out = static_cast<f16*>(d->out) + out_rows * d->out_ld;
    return t;
}

// split-K workspace of the tail launch (the head runs one slice)
static size_t tail_ws_bytes(const c2d_conv_desc* d, int n1) {
    const c2d_conv_desc t = tail_desc(d, n1);
    const long Mt = (long)t.n * t.oh * t.ow;
    const DmaPlan tp = plan_for(Mt, t.cout, t.kpad, t.act, pps_eligible(&t), t.ksize, rr_eligible(&t), panel_eligible(&t));
    return tp.split > 1 ? (size_t)tp.split * Mt * t.cout * sizeof(float) : 0;
}

extern "C" size_t c2d_conv2d_igemm_workspace_size(const c2d_conv_desc* d) {
    if (!d || d->ksize < 1 || d->oh <= 0 || d->ow <= 0 || d->n <= 0 || d->cout <= 0 || d->kpad < 64) return 0;
    if (!dma_eligible(d)) return 0;
    if (d->pro == C2D_PRO_LNFOLD) return 0;   // the panel GEMM, one slice
    const long M = (long)d->n * d->oh * d->ow;
    const DmaPlan pl = plan_for(M, d->cout, d->kpad, d->act, pps_eligible(d), d->ksize, rr_eligible(d), panel_eligible(d));
    if (const int n1 = tail_images(d, pl)) return tail_ws_bytes(d, n1);
    return pl.split > 1 ? (size_t)pl.split * M * d->cout * sizeof(float) : 0;
}

// Rows per GroupNorm-moment block of this descriptor's output as c2d_conv2d_igemm would run it, 0 =
// the plan cannot emit moments.  One slice (after the workspace check the launch makes): the row-ring
// tiles (42: 256 rows, 43 / 44: 128) and the 256 x 320 ping-pong tile 40 (256) through their
// workgroup-image epilogue, which needs a residual or a time embedding; K split: the combine
// (splitk_reduce_gn_kernel, kGnRb rows) at the slice counts it is built for.  Always: no
// quantisation-tail split, act none, 16-B outputs, groups that tile the 320-column block
static bool gn_split_ok(int ks) {   // the slice counts splitk_reduce_gn_kernel is built for
    return ks == 2 || ks == 3 || ks == 4 || ks == 5 || ks == 6 || ks == 8 || ks == 10 || ks == 12 || ks == 15 || ks == 16;
}

static int gn_rows_for(const c2d_conv_desc* d) {
    if (!d || d->gn_groups <= 0 || d->cout % d->gn_groups) return 0;
    const int cpg = d->cout / d->gn_groups;
    if (320 % cpg || d->cout % 320 || d->act != C2D_ACT_NONE) return 0;
    if ((d->out_ld & 7) || (d->resid && (d->resid_ld & 7)) || (d->temb && (d->temb_ld & 7)) || d->out_ld < d->cout) return 0;
    if (((uintptr_t)d->out | (uintptr_t)d->resid | (uintptr_t)d->temb) & 15) return 0;
    if (d->ksize < 1 || d->oh <= 0 || d->ow <= 0 || d->n <= 0 || d->kpad < 64 || !dma_eligible(d)) return 0;
    const long M = (long)d->n * d->oh * d->ow;
    DmaPlan pl = plan_for(M, d->cout, d->kpad, d->act, pps_eligible(d), d->ksize, rr_eligible(d), panel_eligible(d));
    if (pl.id == 50 || pl.id == 70) return 0;   // the persistent / panel tiles never split and emit none
    bool split = false;
    if (pl.split > 1) {
        const size_t need = (size_t)pl.split * M * d->cout * sizeof(float);
        split = d->ws && d->ws_bytes >= need && aligned16(d->ws);   // else the launch runs one slice
    }
    if (d->n >= 2 && tail_images(d, pl)) return 0;
    if (split) {   // the split-K combine emits them (splitk_reduce_gn_kernel), kGnRb-row blocks
        if (pl.id == 42 || pl.id == 43 || pl.id == 44) {   // the row ring's slice count (run_pp16r_t)
            const int ncb = d->c0 / 64, cbs = (pl.nkt + 8) / 9 < 1 ? 1 : ((pl.nkt + 8) / 9 > ncb ? ncb : (pl.nkt + 8) / 9);
            pl.split = (ncb + cbs - 1) / cbs;
        }
        return gn_split_ok(pl.split) && ((long)d->oh * d->ow) % kGnRb == 0 ? kGnRb : 0;
    }
    if (!(d->resid || d->temb)) return 0;   // one slice: only the workgroup-image epilogue emits them
    if (pl.id == 40) return ((long)d->oh * d->ow) % 256 == 0 ? 256 : 0;   // ping-pong 256 x 320 (igemm_pp16.h)
    if (pl.id != 42 && pl.id != 43 && pl.id != 44) return 0;
    return pl.id == 42 ? 256 : 128;
}

extern "C" int c2d_conv2d_gn_rows(const c2d_conv_desc* d) { return gn_rows_for(d); }

extern "C" int c2d_conv2d_igemm_plan(const c2d_conv_desc* d, int* tile_id, int* ksplit) {
    if (!d || !tile_id || !ksplit) return C2D_E_ARG;
    if (d->ksize < 1 || d->oh <= 0 || d->ow <= 0 || d->n <= 0 || d->cout <= 0 || d->kpad < 64) return C2D_E_SHAPE;
    if (d->pro == C2D_PRO_LNFOLD) {   // the panel GEMM or nothing (c2d_conv2d_igemm rejects the rest the same way)
        if (!panel_eligible(d)) return C2D_E_SHAPE;
        *tile_id = 70;
        *ksplit = 1;
        return C2D_OK;
    }
    if (!dma_eligible(d)) {
        *tile_id = 0;
        *ksplit = 1;
        return C2D_OK;
    }
    const long M = (long)d->n * d->oh * d->ow;
    DmaPlan pl = plan_for(M, d->cout, d->kpad, d->act, pps_eligible(d), d->ksize, rr_eligible(d), panel_eligible(d));
    if (pl.split > 1) {
        const size_t need = (size_t)pl.split * M * d->cout * sizeof(float);
        if (!(d->ws && d->ws_bytes >= need && aligned16(d->ws))) pl.split = 1;
    }
    *tile_id = pl.id;
    *ksplit = pl.split;
    return C2D_OK;
}

static int conv_run(const c2d_conv_desc* d, hipStream_t s, const DmaPlan* fixed);

extern "C" int c2d_conv2d_igemm(const c2d_conv_desc* d, void* stream) {
    if (!d || !d->src0 || !d->weight || !d->out) return C2D_E_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (d->gn_mom && gn_rows_for(d) == 0) return C2D_E_SHAPE;   // moments requested of a plan that cannot emit them
    if (d->gn_mom && ((uintptr_t)d->gn_mom & 7)) return C2D_E_ALIGN;
    if (d->n >= 2 && d->ksize >= 1 && d->oh > 0 && d->ow > 0 && d->cout > 0 && d->kpad >= 64 && dma_eligible(d)) {
        const long M = (long)d->n * d->oh * d->ow;
        const DmaPlan pl = plan_for(M, d->cout, d->kpad, d->act, pps_eligible(d), d->ksize, rr_eligible(d), panel_eligible(d));
        if (const int n1 = tail_images(d, pl)) {   // quantisation tail: whole rounds, then the rest
            c2d_conv_desc head = *d;
            head.n = n1;
            const int rc = conv_run(&head, s, &pl);
            if (rc != C2D_OK) return rc;
            const c2d_conv_desc tail = tail_desc(d, n1);
            return conv_run(&tail, s, nullptr);
        }
    }
    return conv_run(d, s, nullptr);
}

// fixed: run this plan (the head of a tail split) instead of planning for d's own M
static int conv_run(const c2d_conv_desc* d, hipStream_t s, const DmaPlan* fixed) {
    if (!d || !d->src0 || !d->weight || !d->out) return C2D_E_ARG;
    if (d->ksize != 1 && d->ksize != 3) return C2D_E_SHAPE;
    if (d->c1 > 0 && !d->src1) return C2D_E_ARG;
    const int cin = d->c0 + d->c1;
    if ((d->c0 & 7) || (d->c1 & 7) || cin <= 0) return C2D_E_SHAPE;
    if (d->kpad & 63) return C2D_E_SHAPE;
    const int ktot = d->ksize * d->ksize * cin;
    if (d->kpad < ktot) return C2D_E_SHAPE;
    if ((d->cout & 3) || d->cout <= 0) return C2D_E_SHAPE;
    if (d->act == C2D_ACT_GEGLU && (d->cout & 31)) return C2D_E_SHAPE;
    if (d->act == C2D_ACT_GEGLU && d->temb) return C2D_E_ARG;
    if (d->act != C2D_ACT_NONE && d->act != C2D_ACT_GEGLU && d->temb) return C2D_E_ARG;
    if ((d->out_ld & 3) || (d->resid && (d->resid_ld & 3)) || (d->temb && (d->temb_ld & 3))) return C2D_E_ALIGN;
    if (!aligned16(d->src0) || (d->src1 && !aligned16(d->src1)) || !aligned16(d->weight)) return C2D_E_ALIGN;
    if (((uintptr_t)d->out & 7) || (d->resid && ((uintptr_t)d->resid & 7)) || (d->temb && ((uintptr_t)d->temb & 7)))
        return C2D_E_ALIGN;
    if (d->bias && ((uintptr_t)d->bias & 15)) return C2D_E_ALIGN;
    if (d->pro == C2D_PRO_GN && (!d->pro_a || !d->pro_b || (cin & 3))) return C2D_E_ARG;
    if (d->pro == C2D_PRO_LN && (!d->pro_a || !d->gamma || !d->beta)) return C2D_E_ARG;
    if (d->pro < 0 || d->pro > 4 || d->act < 0 || d->act > 5) return C2D_E_ARG;
    if (d->pro == C2D_PRO_LNFOLD && !(d->pro_eps > 0.f)) return C2D_E_ARG;   // pro_eps: read only for LNFOLD
    if (d->pro == C2D_PRO_LNFOLD && !panel_eligible(d)) return C2D_E_SHAPE;   // only the panel GEMM folds LN
    if (d->stride != 1 && d->stride != 2) return C2D_E_SHAPE;
    if (d->ksize == 1 && (d->stride != 1 || d->up || d->oh != d->h || d->ow != d->w)) return C2D_E_SHAPE;
    if (d->up && d->stride != 1) return C2D_E_SHAPE;
    // zero-bordered source [n][h + 2][w + 2][c0]: 3x3, stride 1, one source, output h x w
    if (d->src_pad && (d->ksize != 3 || d->stride != 1 || d->up || d->c1 || d->oh != d->h || d->ow != d->w))
        return C2D_E_SHAPE;
    // ... and no prologue: the border is read as data (pad 0), so GN / LN / SiLU would map it to act(shift)
    if (d->src_pad && d->pro != C2D_PRO_NONE) return C2D_E_ARG;

    IgemmParams p;
    p.src0 = (const f16*)d->src0; p.src1 = (const f16*)d->src1;
    p.c0 = d->c0; p.c1 = d->c1; p.cin = cin;
    p.n = d->n; p.h = d->h; p.w = d->w; p.oh = d->oh; p.ow = d->ow;
    p.stride = d->stride; p.up = d->up; p.pad = (d->ksize == 3) ? 1 : 0;
    p.vh = d->up ? 2 * d->h : d->h; p.vw = d->up ? 2 * d->w : d->w;
    if (d->src_pad) {   // a valid 3x3 over the padded image: every kernel's addressing as is, no halo
        p.h = d->h + 2; p.w = d->w + 2; p.vh = p.h; p.vw = p.w; p.pad = 0;
    } else if (d->ksize == 3) {
        int eh = (p.vh + 2 - 3) / d->stride + 1, ew = (p.vw + 2 - 3) / d->stride + 1;
        if (eh != d->oh || ew != d->ow) return C2D_E_SHAPE;
    }
    p.wt = (const f16*)d->weight; p.cout = d->cout; p.kpad = d->kpad; p.ktot = ktot;
    p.pro = d->pro; p.pro_silu = d->pro_silu;
    p.pro_a = d->pro_a; p.pro_b = d->pro_b; p.gamma = d->gamma; p.beta = d->beta;
    p.bias = d->bias; p.act = d->act;
    p.pro_eps = d->pro == C2D_PRO_LNFOLD ? d->pro_eps : 0.f;   // the r5 field: read only when it applies
    p.temb = (const f16*)d->temb; p.temb_ld = d->temb_ld;
    p.resid = (const f16*)d->resid; p.resid_ld = d->resid_ld;
    p.out = (f16*)d->out; p.out_ld = d->out_ld;
    p.M = d->n * d->oh * d->ow;
    p.gn_mom = (float*)d->gn_mom;   // c2d_conv2d_igemm checked gn_rows_for: a one-slice row-ring plan
    p.gn_cpg = d->gn_mom ? d->cout / d->gn_groups : 0;
    if (p.M <= 0) return C2D_OK;

    const int amode = (d->ksize == 1) ? AM_1X1 : ((cin % 64) == 0 ? AM_3X3_FAST : AM_3X3_GEN);
    const bool dma = dma_eligible(d);
    p.ksplit = 1;
    p.nkt = d->kpad / 64;
    p.ws = nullptr;
    p.slab16 = tuning().splitk_f16;
    p.abl = gemm_abl();
    p.lds_epi = (gemm_lds_epi() || !epi_direct_ok(d)) ? 1 : 0;
    p.cmajor = gemm_korder();
    const long t128 = (long)((p.M + 127) / 128) * ((d->cout + 127) / 128);
    if (dma) {
        DmaPlan pl = fixed ? *fixed : plan_for(p.M, d->cout, d->kpad, d->act, pps_eligible(d), d->ksize, rr_eligible(d), panel_eligible(d));
        if (d->pro == C2D_PRO_LNFOLD) pl = {70, 1, d->kpad / 64};   // validated above: panel_eligible
        if (pl.split > 1) {
            const size_t need = (size_t)pl.split * p.M * d->cout * sizeof(float);
            if (d->ws && d->ws_bytes >= need && aligned16(d->ws)) {
                p.ws = (float*)d->ws;
            } else {  // no / short workspace: same tile, one K slice
                pl.split = 1;
                pl.nkt = d->kpad / 64;
            }
        }
        dispatch_dma(p, pl, d->ksize, d->cout, s);
    } else if (t128 < 512) {
        p.gx = (d->cout + 63) / 64; p.gy = (p.M + 63) / 64;
        if (amode == AM_1X1) launch<64, 64, AM_1X1>(p, s);
        else if (amode == AM_3X3_FAST) launch<64, 64, AM_3X3_FAST>(p, s);
        else launch<64, 64, AM_3X3_GEN>(p, s);
    } else {
        p.gx = (d->cout + 127) / 128; p.gy = (p.M + 127) / 128;
        if (amode == AM_1X1) launch<128, 128, AM_1X1>(p, s);
        else if (amode == AM_3X3_FAST) launch<128, 128, AM_3X3_FAST>(p, s);
        else launch<128, 128, AM_3X3_GEN>(p, s);
    }
    return check_launch();
}

#endif  // C2D_PART(0)
