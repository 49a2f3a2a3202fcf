// GroupNorm statistics (folded into per-(image, channel) affine tables) and
// LayerNorm statistics / apply for gfx950.  All HBM-bound: 16-B vector loads,
// per-block LDS reduction, per-block partials reduced by a second kernel.
#include "common.h"
#include <stdlib.h>

namespace c2d {

// ---------------------------------------------------------------- GroupNorm
// ws layout: fp32 [n][nblk][cin][2] per-block shifted moments
// (sum(x-s_g), sum((x-s_g)^2)), written with plain stores and reduced in a
// fixed order by the finalize kernel: no atomics, no memset, bitwise
// reproducible, graph-replay safe.  The per-group shift
// s_g = x[n, pixel 0, first channel of g] keeps the one-pass variance well
// conditioned when |mean| >> std.
__device__ __forceinline__ float gn_read(const f16* s0, const f16* s1, int c0, int c1, size_t pix, int c) {
    return (float)((c < c0) ? s0[pix * c0 + c] : s1[pix * c1 + (c - c0)]);
}

// GP: write per-GROUP pairs ws[n][blk][groups][2] instead (the block's channel totals folded over
// each group's channels in a fixed order, in LDS) -- the input of gn_apply_fold_kernel
template <int CPT, bool GP = false>
__global__ void __launch_bounds__(256) gn_partial_kernel(const f16* __restrict__ s0, const f16* __restrict__ s1,
                                                         int c0, int c1, int hw, int cpg, int rows_per_block,
                                                         float* __restrict__ ws) {
    extern __shared__ __attribute__((aligned(16))) float red[];  // [R][cin*2] (CPT 1), then GP: [cin*2]
    const int cin = c0 + c1, nch = cin >> 3;
    const int n = blockIdx.y;
    const int t = threadIdx.x;
    const int R = (CPT == 1) ? (256 / nch) : 1;
    const int ch_base = (CPT == 1) ? (t % nch) : t;
    const int r0 = (CPT == 1) ? (t / nch) : 0;
    const bool active = (CPT == 1) ? (t < R * nch) : true;
    const int p_begin = blockIdx.x * rows_per_block;
    const int p_end = min(hw, p_begin + rows_per_block);
    const size_t img = (size_t)n * hw;

    float sum[CPT][8], sq[CPT][8], shift[CPT][8];
#pragma unroll
    for (int q = 0; q < CPT; ++q)
#pragma unroll
        for (int i = 0; i < 8; ++i) { sum[q][i] = 0.f; sq[q][i] = 0.f; shift[q][i] = 0.f; }

    if (active) {
        auto ld8 = [&](int pix, int q) {
            const size_t gp = img + pix;
            const int c = (ch_base + q * 256) * 8;
            const f16* ptr = (c < c0) ? (s0 + gp * c0 + c) : (s1 + gp * c1 + (c - c0));
            return *reinterpret_cast<const f16x8*>(ptr);
        };
        auto acc8 = [&](const f16x8& v, int q) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                float d = (float)v[i] - shift[q][i];
                sum[q][i] += d;
                sq[q][i] += d * d;
            }
        };
        // UN pixels per trip, all loads issued before the sums (same per-thread pixel
        // order as one at a time, so the statistics are bit-identical); chunk 0 always
        // exists for an active thread, so CPT = 1 has no per-load branch.  A block owns
        // ~64 rows, i.e. ~11 per thread at 320 channels: eight per trip (not four) halves
        // the HBM round trips of these short-lived blocks, and the first trip's loads are
        // in flight while the per-group shifts load
        constexpr int UN = CPT == 1 ? 8 : 4;
        int pix = p_begin + r0;
        bool first = true;
        for (; pix + (UN - 1) * R < p_end; pix += UN * R) {
            f16x8 v[UN][CPT];
#pragma unroll
            for (int u = 0; u < UN; ++u)
#pragma unroll
                for (int q = 0; q < CPT; ++q)
                    if (q == 0 || ch_base + q * 256 < nch) v[u][q] = ld8(pix + u * R, q);
            if (first) {
#pragma unroll
                for (int q = 0; q < CPT; ++q) {
                    const int ch = ch_base + q * 256;
                    if (ch >= nch) continue;
#pragma unroll
                    for (int i = 0; i < 8; ++i) shift[q][i] = gn_read(s0, s1, c0, c1, img, ((ch * 8 + i) / cpg) * cpg);
                }
                first = false;
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int u = 0; u < UN; ++u)
#pragma unroll
                for (int q = 0; q < CPT; ++q)
                    if (q == 0 || ch_base + q * 256 < nch) acc8(v[u][q], q);
        }
        if (first) {
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                const int ch = ch_base + q * 256;
                if (ch >= nch) continue;
#pragma unroll
                for (int i = 0; i < 8; ++i) shift[q][i] = gn_read(s0, s1, c0, c1, img, ((ch * 8 + i) / cpg) * cpg);
            }
        }
        for (; pix < p_end; pix += R) {
#pragma unroll
            for (int q = 0; q < CPT; ++q)
                if (q == 0 || ch_base + q * 256 < nch) acc8(ld8(pix, q), q);
        }
    }
    if constexpr (GP) {
        // channel totals of the block (fixed row order) -> LDS -> per group, fixed channel order
        float* chs = red + (CPT == 1 ? R * cin * 2 : 0);
        if (CPT == 1) {
            if (active) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    red[(r0 * cin + ch_base * 8 + i) * 2 + 0] = sum[0][i];
                    red[(r0 * cin + ch_base * 8 + i) * 2 + 1] = sq[0][i];
                }
            }
            __syncthreads();
            for (int c = t; c < cin; c += 256) {
                float a = 0.f, b = 0.f;
                for (int r = 0; r < R; ++r) { a += red[(r * cin + c) * 2]; b += red[(r * cin + c) * 2 + 1]; }
                chs[c * 2] = a;
                chs[c * 2 + 1] = b;
            }
        } else {
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                const int ch = ch_base + q * 256;
                if (ch >= nch) continue;
#pragma unroll
                for (int i = 0; i < 8; ++i) { chs[(ch * 8 + i) * 2] = sum[q][i]; chs[(ch * 8 + i) * 2 + 1] = sq[q][i]; }
            }
        }
        __syncthreads();
        const int groups = cin / cpg;
        float* dst = ws + ((size_t)n * gridDim.x + blockIdx.x) * groups * 2;
        for (int g = t; g < groups; g += 256) {
            float a = 0.f, b = 0.f;
            for (int i = 0; i < cpg; ++i) { a += chs[(g * cpg + i) * 2]; b += chs[(g * cpg + i) * 2 + 1]; }
            dst[g * 2] = a;
            dst[g * 2 + 1] = b;
        }
        return;
    }
    // block reduction over the R row-threads sharing a channel chunk
    if (CPT == 1) {
        if (active) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                red[(r0 * cin + ch_base * 8 + i) * 2 + 0] = sum[0][i];
                red[(r0 * cin + ch_base * 8 + i) * 2 + 1] = sq[0][i];
            }
        }
        __syncthreads();
        float* dst = ws + (((size_t)n * gridDim.x + blockIdx.x) * cin) * 2;
        for (int c = t; c < cin; c += 256) {
            float a = 0.f, b = 0.f;
            for (int r = 0; r < R; ++r) { a += red[(r * cin + c) * 2]; b += red[(r * cin + c) * 2 + 1]; }
            dst[c * 2 + 0] = a;
            dst[c * 2 + 1] = b;
        }
    } else {
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int ch = ch_base + q * 256;
            if (ch >= nch) continue;
            float* dst = ws + (((size_t)n * gridDim.x + blockIdx.x) * cin + ch * 8) * 2;
#pragma unroll
            for (int i = 0; i < 8; ++i) { dst[i * 2] = sum[q][i]; dst[i * 2 + 1] = sq[q][i]; }
        }
    }
}

// threads per channel in the finalize: 4 for up to 64 channels per group
__host__ __device__ inline int gn_tpc(int cpg) { return cpg <= 64 ? 4 : (cpg <= 128 ? 2 : 1); }

// grid (n, group chunks): a block owns gpb = 256 / (cpg * tpc) whole groups of one
// image.  tpc threads per channel each sum every tpc-th per-block moment (coalesced
// float2 loads, fixed order, fp64) and combine by a fixed xor butterfly; each group
// then folds its cpg channel totals in fixed order -> mean / rstd -> the
// per-(image, channel) affine tables.  Deterministic, no atomics.
__global__ void __launch_bounds__(256) gn_finalize_kernel(const f16* __restrict__ s0, const f16* __restrict__ s1,
                                                          int c0, int c1, int hw, int groups, int nblk, float eps,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          const float* __restrict__ ws, float* __restrict__ scale,
                                                          float* __restrict__ shift) {
    __shared__ double csum[256], csq[256];
    __shared__ float g_mean[256], g_rstd[256];
    const int cin = c0 + c1, cpg = cin / groups;
    const int tpc = gn_tpc(cpg);
    const int gpb = 256 / (cpg * tpc);
    const int n = blockIdx.x, g0 = blockIdx.y * gpb;
    const int ng = min(gpb, groups - g0);
    const int c_begin = g0 * cpg, nc = ng * cpg;
    const int t = threadIdx.x;
    const int cs = t / tpc, part = t - cs * tpc;
    const size_t img = (size_t)n * hw;
    const float2* wp = reinterpret_cast<const float2*>(ws) + (size_t)n * nblk * cin + c_begin + (cs < nc ? cs : 0);
    double a = 0.0, b = 0.0;
    if (cs < nc) {
        int blk = part;
        for (; blk + 3 * tpc < nblk; blk += 4 * tpc) {
            const float2 v0 = wp[(size_t)blk * cin], v1 = wp[(size_t)(blk + tpc) * cin];
            const float2 v2 = wp[(size_t)(blk + 2 * tpc) * cin], v3 = wp[(size_t)(blk + 3 * tpc) * cin];
            a += (double)v0.x; b += (double)v0.y;
            a += (double)v1.x; b += (double)v1.y;
            a += (double)v2.x; b += (double)v2.y;
            a += (double)v3.x; b += (double)v3.y;
        }
        for (; blk < nblk; blk += tpc) {
            const float2 v = wp[(size_t)blk * cin];
            a += (double)v.x; b += (double)v.y;
        }
    }
    for (int o = 1; o < tpc; o <<= 1) {   // tpc divides 64: a channel's threads share a wave
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
    }
    if (cs < nc && part == 0) {
        csum[cs] = a;
        csq[cs] = b;
    }
    __syncthreads();
    if (t < ng) {
        double a = 0.0, b = 0.0;
        for (int i = 0; i < cpg; ++i) { a += csum[t * cpg + i]; b += csq[t * cpg + i]; }
        const double cnt = (double)hw * cpg;
        const double m1 = a / cnt;
        double var = b / cnt - m1 * m1;
        if (var < 0.0) var = 0.0;
        const float sft = gn_read(s0, s1, c0, c1, img, (g0 + t) * cpg);
        g_mean[t] = (float)(sft + m1);
        g_rstd[t] = (float)(1.0 / sqrt(var + (double)eps));
    }
    __syncthreads();
    if (t < nc) {
        const int c = c_begin + t, gl = t / cpg;
        const float sc = gamma[c] * g_rstd[gl];
        scale[(size_t)n * cin + c] = sc;
        shift[(size_t)n * cin + c] = beta[c] - g_mean[gl] * sc;
    }
}

// GroupNorm apply (+ SiLU): out[m][c] = act(x[m][c] * scale[n][c] + shift[n][c]),
// reading a one- or two-source channel concat and writing the concatenation.
// Grid (pixel blocks, image): a thread owns channel chunks lane_c (+ 256 q) of image
// n, keeps their affine in registers and walks pixels -- no per-chunk index
// divisions or table reloads.  HBM-bound (2 B read + 2 B written / element).
// PAD: the output is the zero-bordered layout [n][h + 2][w + 2][c] (w = pw - 2) that the
// row-ring conv reads (c2d_conv_desc::src_pad): the walk covers the padded pixels, border
// pixels get zeros, interior ones the normalised input.
template <int CPT, bool PAD = false>
__global__ void __launch_bounds__(256) gn_apply_kernel(const f16* __restrict__ s0, const f16* __restrict__ s1, int c0,
                                                       int c1, int hw, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int silu, f16* __restrict__ out,
                                                       int pw = 0) {
    const int cin = c0 + c1, nch = cin >> 3;
    const int L = nch < 256 ? nch : 256, R = 256 / L;
    const int t = threadIdx.x, lane_c = t % L, r0 = t / L;
    if (r0 >= R) return;
    const int n = blockIdx.y;
    const size_t img = (size_t)n * hw;
    float av[CPT][8], bv[CPT][8];
    const f16* src[CPT];
    int ld[CPT], cc[CPT];
    bool on[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const int ch = lane_c + q * 256;
        on[q] = ch < nch;
        cc[q] = (on[q] ? ch : 0) * 8;
        const int c = cc[q];
        src[q] = (c < c0) ? (s0 + c) : (s1 + (c - c0));
        ld[q] = (c < c0) ? c0 : c1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            av[q][i] = scale[(size_t)n * cin + c + i];
            bv[q][i] = shift[(size_t)n * cin + c + i];
        }
    }
    if constexpr (PAD) {
        const int w = pw - 2, ph = hw / w + 2, npix = ph * pw;
        const size_t pimg = (size_t)n * npix;
#pragma unroll 2
        for (int pp = blockIdx.x * R + r0; pp < npix; pp += gridDim.x * R) {
            const int py = pp / pw, px = pp - py * pw;
            const bool inner = py >= 1 && py < ph - 1 && px >= 1 && px < pw - 1;
            const size_t gp = img + (inner ? (py - 1) * w + (px - 1) : 0);
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                if (!on[q]) continue;
                f16x8 o = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
                if (inner) {
                    const f16x8 v = *reinterpret_cast<const f16x8*>(src[q] + gp * ld[q]);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float y = fmaf((float)v[j], av[q][j], bv[q][j]);
                        if (silu) y = y * __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                        o[j] = (f16)y;
                    }
                }
                *reinterpret_cast<f16x8*>(out + (pimg + pp) * cin + cc[q]) = o;
            }
        }
        return;
    }
#pragma unroll 4
    for (int pix = blockIdx.x * R + r0; pix < hw; pix += gridDim.x * R) {
        const size_t gp = img + pix;
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            if (!on[q]) continue;
            const f16x8 v = *reinterpret_cast<const f16x8*>(src[q] + gp * ld[q]);
            f16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float y = fmaf((float)v[j], av[q][j], bv[q][j]);
                if (silu) y = y * __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                o[j] = (f16)y;
            }
            *reinterpret_cast<f16x8*>(out + gp * cin + cc[q]) = o;
        }
    }
}

// GroupNorm apply that folds the statistics itself (no finalize launch): every workgroup of
// image n first folds the nblk per-group pairs gn_partial_kernel<., true> wrote (a few KB,
// L2-resident; 256 / groups threads per group, fixed order, fp64), forms mean / rstd and
// gn_finalize_kernel's per-channel affine for its own channels, then walks its pixels as
// gn_apply_kernel does (PAD: the zero-bordered layout).  Same statistics in every workgroup of
// an image: the fold order does not depend on the workgroup.
//
// MOM: ws holds {mean, M2} per (image, block of mrows pixels, group) written by the producing conv
// (c2d_conv_desc::gn_mom) instead of shifted sums: each of the `parts` threads of a group sums every
// parts-th block's shifted mean, its square and its M2 (fp64), then the group's thread adds the parts in
// order and forms the group's mean and M2 (equal block counts: no per-block divisions).  Deterministic;
// no pass over the source for statistics.
template <int CPT, bool PAD, bool MOM = false>
__global__ void __launch_bounds__(256) gn_apply_fold_kernel(const f16* __restrict__ s0, const f16* __restrict__ s1,
                                                            int c0, int c1, int hw, int cpg, int nblk, float eps,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ ws, int silu,
                                                            f16* __restrict__ out, int pw = 0, int mrows = 0) {
    __shared__ double dacc[MOM ? 768 : 512];   // [256][2] fold partials (MOM: [256][3] count, mean, M2)
    __shared__ float gmr[512];     // [groups][2] mean, rstd (groups <= 256)
    const int cin = c0 + c1, nch = cin >> 3, groups = cin / cpg;
    const int L = nch < 256 ? nch : 256, R = 256 / L;
    const int t = threadIdx.x, lane_c = t % L, r0 = t / L;
    const int n = blockIdx.y;
    const size_t img = (size_t)n * hw;
    const int parts = 256 / groups;
    if constexpr (MOM) {
        // equal counts nb per block: mean = s + S1 / K, M2 = Q + nb (S2 - S1^2 / K) with S1, S2 the sums of
        // (mean_k - s), (mean_k - s)^2 over the K blocks and Q the sum of their M2; s = block 0's mean
        // (the blocks' means sit close together, so the shifted sums stay well conditioned in fp64)
        const double nb = (double)mrows * cpg;
        if (t < parts * groups) {
            const int g = t % groups, pt = t / groups;
            const float2* wp = reinterpret_cast<const float2*>(ws) + (size_t)n * nblk * groups + g;
            const double sh = (double)wp[0].x;
            double a = 0.0, b = 0.0, qq = 0.0;
            for (int k = pt; k < nblk; k += parts) {
                const float2 v = wp[(size_t)k * groups];
                const double d = (double)v.x - sh;
                a += d;
                b += d * d;
                qq += (double)v.y;
            }
            dacc[t * 3] = a;
            dacc[t * 3 + 1] = b;
            dacc[t * 3 + 2] = qq;
        }
        __syncthreads();
        if (t < groups) {
            double a = 0.0, b = 0.0, qq = 0.0;
            for (int pt = 0; pt < parts; ++pt) {
                const int u = (pt * groups + t) * 3;
                a += dacc[u];
                b += dacc[u + 1];
                qq += dacc[u + 2];
            }
            const float2* wp = reinterpret_cast<const float2*>(ws) + (size_t)n * nblk * groups + t;
            const double K = (double)nblk;
            double var = (qq + nb * (b - a * a / K)) / (K * nb);
            if (var < 0.0) var = 0.0;
            gmr[t * 2] = (float)((double)wp[0].x + a / K);
            gmr[t * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
        }
    } else {
    if (t < parts * groups) {
        const int g = t % groups, pt = t / groups;
        const float2* wp = reinterpret_cast<const float2*>(ws) + (size_t)n * nblk * groups + g;
        double a = 0.0, b = 0.0;
        int k = pt;
        for (; k + 3 * parts < nblk; k += 4 * parts) {
            const float2 v0 = wp[(size_t)k * groups], v1 = wp[(size_t)(k + parts) * groups];
            const float2 v2 = wp[(size_t)(k + 2 * parts) * groups], v3 = wp[(size_t)(k + 3 * parts) * groups];
            a += (double)v0.x; b += (double)v0.y;
            a += (double)v1.x; b += (double)v1.y;
            a += (double)v2.x; b += (double)v2.y;
            a += (double)v3.x; b += (double)v3.y;
        }
        for (; k < nblk; k += parts) {
            const float2 v = wp[(size_t)k * groups];
            a += (double)v.x; b += (double)v.y;
        }
        dacc[t * 2] = a;
        dacc[t * 2 + 1] = b;
    }
    __syncthreads();
    if (t < groups) {
        double a = 0.0, b = 0.0;
        for (int pt = 0; pt < parts; ++pt) { a += dacc[(pt * groups + t) * 2]; b += dacc[(pt * groups + t) * 2 + 1]; }
        const double cnt = (double)hw * cpg;
        const double m1 = a / cnt;
        double var = b / cnt - m1 * m1;
        if (var < 0.0) var = 0.0;
        gmr[t * 2] = (float)(gn_read(s0, s1, c0, c1, img, t * cpg) + m1);
        gmr[t * 2 + 1] = (float)(1.0 / sqrt(var + (double)eps));
    }
    }
    __syncthreads();
    if (r0 >= R) return;
    float av[CPT][8], bv[CPT][8];
    const f16* src[CPT];
    int ld[CPT], cc[CPT];
    bool on[CPT];
#pragma unroll
    for (int q = 0; q < CPT; ++q) {
        const int ch = lane_c + q * 256;
        on[q] = ch < nch;
        cc[q] = (on[q] ? ch : 0) * 8;
        const int c = cc[q];
        src[q] = (c < c0) ? (s0 + c) : (s1 + (c - c0));
        ld[q] = (c < c0) ? c0 : c1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int gl = (c + i) / cpg;
            const float sc = gamma[c + i] * gmr[gl * 2 + 1];
            av[q][i] = sc;
            bv[q][i] = beta[c + i] - gmr[gl * 2] * sc;
        }
    }
    if constexpr (PAD) {
        const int w = pw - 2, ph = hw / w + 2, npix = ph * pw;
        const size_t pimg = (size_t)n * npix;
#pragma unroll 2
        for (int pp = blockIdx.x * R + r0; pp < npix; pp += gridDim.x * R) {
            const int py = pp / pw, px = pp - py * pw;
            const bool inner = py >= 1 && py < ph - 1 && px >= 1 && px < pw - 1;
            const size_t gp = img + (inner ? (py - 1) * w + (px - 1) : 0);
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                if (!on[q]) continue;
                f16x8 o = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
                if (inner) {
                    const f16x8 v = *reinterpret_cast<const f16x8*>(src[q] + gp * ld[q]);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float y = fmaf((float)v[j], av[q][j], bv[q][j]);
                        if (silu) y = y * __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                        o[j] = (f16)y;
                    }
                }
                *reinterpret_cast<f16x8*>(out + (pimg + pp) * cin + cc[q]) = o;
            }
        }
        return;
    }
#pragma unroll 4
    for (int pix = blockIdx.x * R + r0; pix < hw; pix += gridDim.x * R) {
        const size_t gp = img + pix;
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            if (!on[q]) continue;
            const f16x8 v = *reinterpret_cast<const f16x8*>(src[q] + gp * ld[q]);
            f16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float y = fmaf((float)v[j], av[q][j], bv[q][j]);
                if (silu) y = y * __builtin_amdgcn_rcpf(1.0f + __expf(-y));
                o[j] = (f16)y;
            }
            *reinterpret_cast<f16x8*>(out + gp * cin + cc[q]) = o;
        }
    }
}

// Single-launch GroupNorm (+ SiLU) for small images: one workgroup owns image n
// and a chunk of CB channels (whole groups, CB % 8 == 0); L = CB / 8 lanes per
// pixel row, R = NT / L rows.  Pass 1 accumulates per-thread shifted moments
// (fp32), the block folds them in a fixed order (fp64) -> per-group mean / rstd
// -> per-channel affine in LDS; pass 2 re-reads the slab (L2 / MALL resident)
// and writes act(x * scale + shift).  Deterministic; replaces partial + finalize
// + apply (three launches of a few microseconds each) where the image is small.
// NT > 256 folds its rows into the 256-row reduction buffer in NT / 256 (+1) fixed-order
// phases (row r0 adds into slot r0 % R1 after rows r0 - R1, r0 - 2 R1, ...).  A 1024-thread
// form for few large images (c2's N = 2 at 64^2 / 32^2, where 256 threads walk ~80 pixel rows
// each) measured 2x slower than partial + finalize + apply there (13.5 -> 29.7 us at
// 64^2 x 320, profiles/r03h_ab.txt: 2 x C / CB workgroups cannot pull the bytes); only
// NT = 256 is launched.
template <int NT>
__global__ void __launch_bounds__(NT) gn_fused_kernel(const f16* __restrict__ s0, const f16* __restrict__ s1, int c0,
                                                      int c1, int hw, int cpg, int cb, float eps,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      int silu, f16* __restrict__ out) {
    __shared__ float red[2 * 2048];            // [R1][CB][2], R1 * CB <= 256 * 8
    __shared__ double gsum[256], gsq[256];     // per channel of the chunk (CB <= 256)
    __shared__ float aff[2 * 256];             // scale | shift per channel of the chunk
    const int cin = c0 + c1;
    const int L = cb >> 3, R = NT / L, R1 = 256 / L;
    const int n = blockIdx.y, cbase = blockIdx.x * cb;
    const int t = threadIdx.x, lane_c = t % L, r0 = t / L;
    const bool active = r0 < R && cbase + lane_c * 8 < cin;
    const int c = cbase + lane_c * 8;
    const size_t img = (size_t)n * hw;
    const f16* src = (c < c0) ? (s0 + c) : (s1 + (c - c0));
    const int ld = (c < c0) ? c0 : c1;
    float sh[8], sum[8], sq[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { sum[i] = 0.f; sq[i] = 0.f; sh[i] = 0.f; }
    if (active) {
#pragma unroll
        for (int i = 0; i < 8; ++i) sh[i] = gn_read(s0, s1, c0, c1, img, ((c + i) / cpg) * cpg);
#pragma unroll 4
        for (int pix = r0; pix < hw; pix += R) {
            const f16x8 v = *reinterpret_cast<const f16x8*>(src + (img + pix) * ld);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float d = (float)v[i] - sh[i];
                sum[i] += d;
                sq[i] += d * d;
            }
        }
    }
    const int nph = (R + R1 - 1) / R1;
    for (int ph = 0; ph < nph; ++ph) {
        if (r0 < R && r0 / R1 == ph) {
            float* dst = red + ((r0 - ph * R1) * cb + lane_c * 8) * 2;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if (ph == 0) {
                    dst[i * 2] = sum[i];
                    dst[i * 2 + 1] = sq[i];
                } else {
                    dst[i * 2] += sum[i];
                    dst[i * 2 + 1] += sq[i];
                }
            }
        }
        __syncthreads();
    }
    const int rs = R < R1 ? R : R1;   // reduction slots written
    if (t < cb) {
        double a = 0.0, b = 0.0;
        for (int r = 0; r < rs; ++r) { a += (double)red[(r * cb + t) * 2]; b += (double)red[(r * cb + t) * 2 + 1]; }
        gsum[t] = a;
        gsq[t] = b;
    }
    __syncthreads();
    if (t < cb && cbase + t < cin) {
        const int gl = t / cpg;                  // group within the chunk (chunks hold whole groups)
        double a = 0.0, b = 0.0;
        for (int i = 0; i < cpg; ++i) { a += gsum[gl * cpg + i]; b += gsq[gl * cpg + i]; }
        const double cnt = (double)hw * cpg;
        const double m1 = a / cnt;
        double var = b / cnt - m1 * m1;
        if (var < 0.0) var = 0.0;
        const float mean = (float)(gn_read(s0, s1, c0, c1, img, cbase + gl * cpg) + m1);
        const float rstd = (float)(1.0 / sqrt(var + (double)eps));
        const float scl = gamma[cbase + t] * rstd;
        aff[t] = scl;
        aff[256 + t] = beta[cbase + t] - mean * scl;
    }
    __syncthreads();
    if (!active) return;
    float av[8], bv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { av[i] = aff[lane_c * 8 + i]; bv[i] = aff[256 + lane_c * 8 + i]; }
#pragma unroll 4
    for (int pix = r0; pix < hw; pix += R) {
        const f16x8 v = *reinterpret_cast<const f16x8*>(src + (img + pix) * ld);
        f16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            float y = fmaf((float)v[i], av[i], bv[i]);
            if (silu) y = y * __builtin_amdgcn_rcpf(1.0f + __expf(-y));
            o[i] = (f16)y;
        }
        *reinterpret_cast<f16x8*>(out + (img + pix) * cin + c) = o;
    }
}

// ---------------------------------------------------------------- LayerNorm
// one wave per row, up to 4 chunks (32 values) per lane in registers: exact
// two-pass mean / variance.
template <int NCH, bool APPLY>
__global__ void __launch_bounds__(256) ln_kernel(const f16* __restrict__ x, int m, int c, int ld, float eps,
                                                 float* __restrict__ stats, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, f16* __restrict__ out, int out_ld) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= m) return;
    const int nch = c >> 3;
    const f16* xr = x + (size_t)row * ld;
    f16x8 v[NCH];
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
        const int ch = lane + q * 64;
        if (ch < nch) {
            v[q] = *reinterpret_cast<const f16x8*>(xr + ch * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) s += (float)v[q][i];
        }
    }
    const float mean = wave_sum(s) / (float)c;
    float s2 = 0.f;
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
        const int ch = lane + q * 64;
        if (ch < nch) {
#pragma unroll
            for (int i = 0; i < 8; ++i) { float d = (float)v[q][i] - mean; s2 += d * d; }
        }
    }
    const float rstd = rsqrtf(wave_sum(s2) / (float)c + eps);
    if (!APPLY) {
        if (lane == 0) { stats[(size_t)row * 2] = mean; stats[(size_t)row * 2 + 1] = rstd; }
        return;
    }
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
        const int ch = lane + q * 64;
        if (ch < nch) {
            f16x8 o;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int cc = ch * 8 + i;
                o[i] = (f16)(((float)v[q][i] - mean) * rstd * gamma[cc] + beta[cc]);
            }
            *reinterpret_cast<f16x8*>(out + (size_t)row * out_ld + ch * 8) = o;
        }
    }
}

// LayerNorm + apply with LPR lanes per row and CPL 16-B chunks per lane (the row's
// C = 8 * LPR * CPL channels in registers): 64 / LPR rows per wave, exact two-pass
// mean / variance over an LPR-lane xor butterfly, the lane's gamma / beta loaded once
// and kept across its rows.  The one-wave-per-row kernel left 24 of 64 lanes idle at
// C = 320 and paid two full-wave reductions per 640-B row.
template <int LPR, int CPL>
__global__ void __launch_bounds__(256) ln_rows_kernel(const f16* __restrict__ x, int m, int ld, float eps,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      f16* __restrict__ out, int out_ld) {
    constexpr int C = 8 * LPR * CPL;
    constexpr int RPW = 64 / LPR;                    // rows per wave
    const int lane = threadIdx.x & 63;
    const int sub = lane % LPR, rw = lane / LPR;
    const int wave_g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nwaves = gridDim.x * 4;
    float g[CPL][8], b[CPL][8];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = (sub + k * LPR) * 8;
#pragma unroll
        for (int i = 0; i < 8; i += 4) {
            const float4 gg = *reinterpret_cast<const float4*>(gamma + c + i);
            const float4 bb = *reinterpret_cast<const float4*>(beta + c + i);
            g[k][i] = gg.x; g[k][i + 1] = gg.y; g[k][i + 2] = gg.z; g[k][i + 3] = gg.w;
            b[k][i] = bb.x; b[k][i + 1] = bb.y; b[k][i + 2] = bb.z; b[k][i + 3] = bb.w;
        }
    }
    for (int row0 = wave_g * RPW; row0 < m; row0 += nwaves * RPW) {
        const int row = row0 + rw;
        const bool ok = row < m;
        const f16* xr = x + (size_t)(ok ? row : 0) * ld;
        f16x8 v[CPL];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            v[k] = *reinterpret_cast<const f16x8*>(xr + (sub + k * LPR) * 8);
#pragma unroll
            for (int i = 0; i < 8; ++i) s += (float)v[k][i];
        }
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) s += __shfl_xor(s, o);
        const float mean = s * (1.0f / C);
        float s2 = 0.f;
#pragma unroll
        for (int k = 0; k < CPL; ++k)
#pragma unroll
            for (int i = 0; i < 8; ++i) { const float d = (float)v[k][i] - mean; s2 += d * d; }
#pragma unroll
        for (int o = 1; o < LPR; o <<= 1) s2 += __shfl_xor(s2, o);
        const float rstd = rsqrtf(s2 * (1.0f / C) + eps);
        if (!ok) continue;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            f16x8 o;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (f16)(((float)v[k][i] - mean) * rstd * g[k][i] + b[k][i]);
            *reinterpret_cast<f16x8*>(out + (size_t)row * out_ld + (sub + k * LPR) * 8) = o;
        }
    }
}

// C = 8 * LPR * CPL for LPR in {4, 8, 16, 32}, CPL in {3, 5}: the UNet (320 / 640 / 1280)
// and HTSAT (96 / 192 / 384 / 768) widths; returns 1 (not launched) when the shape
// needs the generic kernel, else the launch status
static int ln_rows_launch(const void* x, int m, int c, int ld, float eps, const float* gamma, const float* beta,
                          void* out, int out_ld, hipStream_t s) {
    if ((ld & 7) || (out_ld & 7) || !aligned16(gamma) || !aligned16(beta)) return 1;
    const int nch = c >> 3;
    int cpl = 0, lpr = 0;
    for (int cp : {5, 3}) {
        if (nch % cp) continue;
        const int l = nch / cp;
        if (l == 4 || l == 8 || l == 16 || l == 32) { cpl = cp; lpr = l; break; }
    }
    if (!cpl) return 1;
    const int rows_per_block = 4 * (64 / lpr);
    long want = ((long)m + rows_per_block - 1) / rows_per_block;
    const unsigned blocks = (unsigned)(want < 4096 ? want : 4096);
#define C2D_LNR(L, P)                                                                                            \
    if (lpr == L && cpl == P) {                                                                                  \
        hipLaunchKernelGGL((ln_rows_kernel<L, P>), dim3(blocks), dim3(256), 0, s, (const f16*)x, m, ld, eps, gamma, \
                           beta, (f16*)out, out_ld);                                                             \
        return check_launch();                                                                                   \
    }
    C2D_LNR(4, 3) C2D_LNR(8, 3) C2D_LNR(16, 3) C2D_LNR(32, 3)
    C2D_LNR(4, 5) C2D_LNR(8, 5) C2D_LNR(16, 5) C2D_LNR(32, 5)
#undef C2D_LNR
    return 1;
}

template <bool APPLY>
static int ln_dispatch(const void* x, int m, int c, int ld, float eps, float* stats, const float* gamma,
                       const float* beta, void* out, int out_ld, hipStream_t s) {
    if (APPLY) {
        const int rc = ln_rows_launch(x, m, c, ld, eps, gamma, beta, out, out_ld, s);
        if (rc != 1) return rc;
    }
    const int nch = c >> 3;
    dim3 grid((m + 3) / 4);
    if (nch <= 64)
        hipLaunchKernelGGL((ln_kernel<1, APPLY>), grid, dim3(256), 0, s, (const f16*)x, m, c, ld, eps, stats, gamma, beta, (f16*)out, out_ld);
    else if (nch <= 128)
        hipLaunchKernelGGL((ln_kernel<2, APPLY>), grid, dim3(256), 0, s, (const f16*)x, m, c, ld, eps, stats, gamma, beta, (f16*)out, out_ld);
    else if (nch <= 256)
        hipLaunchKernelGGL((ln_kernel<4, APPLY>), grid, dim3(256), 0, s, (const f16*)x, m, c, ld, eps, stats, gamma, beta, (f16*)out, out_ld);
    else if (nch <= 512)
        hipLaunchKernelGGL((ln_kernel<8, APPLY>), grid, dim3(256), 0, s, (const f16*)x, m, c, ld, eps, stats, gamma, beta, (f16*)out, out_ld);
    else
        return C2D_E_SHAPE;
    return check_launch();
}

}  // namespace c2d

using namespace c2d;

// target partial-block count of a launch (C2D_TUNE_GN_BLOCKS, A/B only).  512: 64^2 x 320 GN
// 30.5 -> 29.3 us, 32^2 x 640 23.4 -> 20.6 us vs 1024 (graph-replayed, same box; 2048 slower)
static int gn_target_blocks() { return tuning().gn_blocks; }

// rows (pixels) per partial block: about gn_target_blocks() blocks over the whole launch,
// at least one full pass of the block's row-threads, at most 128
// apply workgroups per launch (C2D_TUNE_GN_APPLY_BLOCKS, A/B only; default 2048)
static int gn_apply_blocks() { return tuning().gn_apply_blocks; }

// rows per partial block: about gn_target_blocks() blocks over the launch, but at most
// ~32 per image -- the finalize folds an image's partials serially (fixed order), so at
// small N (c2: N = 2, 64^2) 228 blocks per image made it a 9.2-us latency chain per call
static int gn_rows_per_block(int n, int c, int hw, int cap = 32) {
    const int nch = c >> 3;
    const int r = nch <= 256 ? 256 / nch : 1;
    const long tb = gn_target_blocks();
    long want = ((long)n * hw + tb - 1) / tb;
    if (want < (hw + cap - 1) / cap) want = (hw + cap - 1) / cap;
    if (want < r) want = r;
    if (want > 128) want = 128;
    return (int)((want + r - 1) / r * r);
}

static int gn_blocks(int n, int c, int hw, int cap = 32) {
    const int rpb = gn_rows_per_block(n, c, hw, cap);
    return (hw + rpb - 1) / rpb;
}

extern "C" size_t c2d_groupnorm_workspace_size(int n, int c, int hw) {
    if (n <= 0 || c <= 0 || hw <= 0) return 0;
    return (size_t)n * gn_blocks(n, c, hw) * c * 2 * sizeof(float);
}

extern "C" int c2d_groupnorm_stats(const void* src0, const void* src1, int c0, int c1, int n, int hw, int groups,
                                   float eps, const float* gamma, const float* beta, float* scale, float* shift,
                                   void* ws, void* stream) {
    if (!src0 || !gamma || !beta || !scale || !shift || !ws) return C2D_E_ARG;
    if (c1 > 0 && !src1) return C2D_E_ARG;
    const int cin = c0 + c1;
    if ((c0 & 7) || (c1 & 7) || cin <= 0 || groups <= 0 || cin % groups) return C2D_E_SHAPE;
    if (cin / groups > 256 || n <= 0 || hw <= 0) return C2D_E_SHAPE;
    if (!aligned16(src0) || (src1 && !aligned16(src1))) return C2D_E_ALIGN;
    hipStream_t s = (hipStream_t)stream;
    const int nch = cin >> 3;
    const int cpg = cin / groups;
    const int rows_per_block = gn_rows_per_block(n, cin, hw);
    const int nblk = gn_blocks(n, cin, hw);
    dim3 grid(nblk, n);
    if (nch <= 256) {
        const int R = 256 / nch;
        const size_t lds = (size_t)R * cin * 2 * sizeof(float);
        hipLaunchKernelGGL((gn_partial_kernel<1>), grid, dim3(256), lds, s, (const f16*)src0, (const f16*)src1, c0, c1,
                           hw, cpg, rows_per_block, (float*)ws);
    } else {
        hipLaunchKernelGGL((gn_partial_kernel<2>), grid, dim3(256), 0, s, (const f16*)src0, (const f16*)src1, c0, c1,
                           hw, cpg, rows_per_block, (float*)ws);
    }
    const int gpb = 256 / (cpg * gn_tpc(cpg));
    hipLaunchKernelGGL(gn_finalize_kernel, dim3(n, (groups + gpb - 1) / gpb), dim3(256), 0, s, (const f16*)src0, (const f16*)src1, c0, c1, hw,
                       groups, nblk, eps, gamma, beta, (const float*)ws, scale, shift);
    return check_launch();
}

extern "C" int c2d_layernorm_stats(const void* x, int m, int c, int ld, float eps, float* stats, void* stream) {
    if (!x || !stats) return C2D_E_ARG;
    if ((c & 7) || (ld & 7) || c <= 0) return C2D_E_SHAPE;
    if (!aligned16(x)) return C2D_E_ALIGN;
    if (m <= 0) return C2D_OK;
    return ln_dispatch<false>(x, m, c, ld, eps, stats, nullptr, nullptr, nullptr, 0, (hipStream_t)stream);
}

extern "C" int c2d_layernorm(const void* x, int m, int c, int ld, float eps, const float* gamma, const float* beta,
                             void* out, int out_ld, void* stream) {
    if (!x || !gamma || !beta || !out) return C2D_E_ARG;
    if ((c & 7) || (ld & 7) || (out_ld & 7) || c <= 0) return C2D_E_SHAPE;
    if (!aligned16(x) || !aligned16(out)) return C2D_E_ALIGN;
    if (m <= 0) return C2D_OK;
    return ln_dispatch<true>(x, m, c, ld, eps, nullptr, gamma, beta, out, out_ld, (hipStream_t)stream);
}

extern "C" int c2d_groupnorm_apply(const void* src0, const void* src1, int c0, int c1, int n, int hw,
                                   const float* scale, const float* shift, int silu, void* out, void* stream) {
    if (!src0 || !scale || !shift || !out) return C2D_E_ARG;
    if (c1 > 0 && !src1) return C2D_E_ARG;
    if ((c0 & 7) || (c1 & 7) || c0 + c1 <= 0 || n <= 0 || hw <= 0) return C2D_E_SHAPE;
    if (!aligned16(src0) || (src1 && !aligned16(src1)) || !aligned16(out) || !aligned16(scale) || !aligned16(shift))
        return C2D_E_ALIGN;
    const int nch = (c0 + c1) >> 3;
    if (nch > 512) return C2D_E_SHAPE;
    const int L = nch < 256 ? nch : 256, R = 256 / L;
    // about gn_apply_blocks() workgroups over the launch, each at least one pass of its rows
    int bx = (gn_apply_blocks() + n - 1) / n;
    const int maxb = (hw + R - 1) / R;
    if (bx > maxb) bx = maxb;
    if (bx < 1) bx = 1;
    if (nch <= 256)
        hipLaunchKernelGGL(gn_apply_kernel<1>, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, (const f16*)src0,
                           (const f16*)src1, c0, c1, hw, scale, shift, silu, (f16*)out);
    else
        hipLaunchKernelGGL(gn_apply_kernel<2>, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, (const f16*)src0,
                           (const f16*)src1, c0, c1, hw, scale, shift, silu, (f16*)out);
    return check_launch();
}

// channels per fused-GN workgroup: whole groups, a multiple of 8, <= 256, as few as
// keep the launch at >= 256 workgroups; 0 when the shape does not fit the kernel
static int gn_fused_cb(int n, int cin, int groups) {
    const int cpg = cin / groups;
    int u = cpg;
    while (u % 8) u += cpg;                       // lcm(cpg, 8)
    if (u > 256) return 0;
    int cb = u;
    while (cb * 2 <= 256 && cin % (cb * 2) == 0 && (long)n * (cin / (cb * 2)) >= 256) cb *= 2;
    return cb;
}

// pixels per image up to which the single-launch kernel is used (C2D_TUNE_GN_FUSED_HW).
// Graph-replayed per call at N = 16 (scripts/bench_norm_graph.py): 8^2 x 1280
// 16.8 -> 6.2 us, 16^2 x 1280 21.3 -> 13.0 us, but 32^2 x 640 23.1 -> 26.6 us
// (40-channel chunks read 80-B row pieces over 1024 pixels) and 64^2 2-5x slower.
static int gn_fused_max_hw() { return tuning().gn_fused_hw; }

static bool gn_use_fused(int n, int cin, int hw, int groups) {
    return gn_fused_cb(n, cin, groups) > 0 && hw <= gn_fused_max_hw();
}


// partial (per-group pairs) + apply-with-fold: two launches where c2d_groupnorm_stats +
// c2d_groupnorm_apply take three (C2D_TUNE_GN_FOLD=0 restores those, A/B only).  Needs groups <= 256.
// Every apply workgroup folds all its image's partial pairs (nblk x groups x 8 B).  Rows per
// partial block stop at 128, so a 512^2 VAE image has 2048 blocks (512 KB of L2 reads per apply
// workgroup at 32 groups); measured against the three-launch path (parallel finalize +
// plain apply) on the VAE shapes at 8 images the fold is still faster -- 256^2 x 512 318.8 vs
// 336.3 us, 512^2 x 256 644.1 vs 698.1 us, 512^2 x 128 356.9 vs 392.1 us, graph-replayed on one box
// (profiles/r05_gn_vae_fold_ab.txt) -- so every shape within the kernel's limits folds.
static bool gn_use_fold(int n, int cin, int hw, int groups) {
    (void)n; (void)hw;
    return tuning().gn_fold != 0 && groups <= 256 && (cin >> 3) <= 512;
}

static int gn_fold_run(const void* src0, const void* src1, int c0, int c1, int n, int hw, int pw, int groups,
                       float eps, const float* gamma, const float* beta, int silu, void* out, void* ws, hipStream_t s) {
    const int cin = c0 + c1, nch = cin >> 3, cpg = cin / groups;
    const int cap = tuning().gn_fold_cap;   // partial blocks per image (the apply's fold is parallel)
    const int rows_per_block = gn_rows_per_block(n, cin, hw, cap);
    const int nblk = gn_blocks(n, cin, hw, cap);
    const dim3 pgrid(nblk, n);
    if (nch <= 256) {
        const size_t lds = ((size_t)(256 / nch) * cin * 2 + (size_t)cin * 2) * sizeof(float);
        hipLaunchKernelGGL((gn_partial_kernel<1, true>), pgrid, dim3(256), lds, s, (const f16*)src0, (const f16*)src1,
                           c0, c1, hw, cpg, rows_per_block, (float*)ws);
    } else {
        hipLaunchKernelGGL((gn_partial_kernel<2, true>), pgrid, dim3(256), (size_t)cin * 2 * sizeof(float), s,
                           (const f16*)src0, (const f16*)src1, c0, c1, hw, cpg, rows_per_block, (float*)ws);
    }
    const int L = nch < 256 ? nch : 256, R = 256 / L;
    const int npix = pw ? (hw / (pw - 2) + 2) * pw : hw;
    // small batches: fewer, longer apply workgroups (each folds the pairs first): 1024 vs 2048 made
    // c2's norms 1-2 us faster and c2 0.3079 -> 0.3065 s; c3's N = 16 keeps 2048 (equal per call, the
    // bench 0.1-0.2 % either way; profiles/r04_gn_two_launch_ab.txt)
    int bx = ((n < 8 ? tuning().gn_fold_apply_blocks : gn_apply_blocks()) + n - 1) / n;
    const int maxb = (npix + R - 1) / R;
    if (bx > maxb) bx = maxb;
    if (bx < 1) bx = 1;
    const dim3 agrid(bx, n);
#define C2D_GNF(C, PD)                                                                                           \
    hipLaunchKernelGGL((gn_apply_fold_kernel<C, PD>), agrid, dim3(256), 0, s, (const f16*)src0, (const f16*)src1, c0, \
                       c1, hw, cpg, nblk, eps, gamma, beta, (const float*)ws, silu, (f16*)out, pw)
    if (nch <= 256) {
        if (pw) C2D_GNF(1, true); else C2D_GNF(1, false);
    } else {
        if (pw) C2D_GNF(2, true); else C2D_GNF(2, false);
    }
#undef C2D_GNF
    return check_launch();
}

extern "C" int c2d_groupnorm_moments(const void* src, int c, int n, int hw, int groups, float eps, const float* gamma,
                                     const float* beta, int silu, const float* mom, int rows, int pw, void* out,
                                     void* stream) {
    if (!src || !gamma || !beta || !mom || !out) return C2D_E_ARG;
    if ((c & 7) || c <= 0 || (c >> 3) > 512 || groups <= 0 || groups > 256 || c % groups || n <= 0 || hw <= 0)
        return C2D_E_SHAPE;
    if (rows <= 0 || hw % rows) return C2D_E_SHAPE;
    if (pw && (pw < 3 || hw % (pw - 2))) return C2D_E_SHAPE;
    if (!aligned16(src) || !aligned16(out) || ((uintptr_t)mom & 7)) return C2D_E_ALIGN;
    const int nch = c >> 3, cpg = c / groups, nblk = hw / rows;
    const int L = nch < 256 ? nch : 256, R = 256 / L;
    const int npix = pw ? (hw / (pw - 2) + 2) * pw : hw;
    int bx = ((n < 8 ? tuning().gn_fold_apply_blocks : gn_apply_blocks()) + n - 1) / n;   // as gn_fold_run
    const int maxb = (npix + R - 1) / R;
    if (bx > maxb) bx = maxb;
    if (bx < 1) bx = 1;
    const dim3 agrid(bx, n);
    hipStream_t s = (hipStream_t)stream;
#define C2D_GNM(C, PD)                                                                                            \
    hipLaunchKernelGGL((gn_apply_fold_kernel<C, PD, true>), agrid, dim3(256), 0, s, (const f16*)src, (const f16*)nullptr, \
                       c, 0, hw, cpg, nblk, eps, gamma, beta, mom, silu, (f16*)out, pw, rows)
    if (nch <= 256) {
        if (pw) C2D_GNM(1, true); else C2D_GNM(1, false);
    } else {
        if (pw) C2D_GNM(2, true); else C2D_GNM(2, false);
    }
#undef C2D_GNM
    return check_launch();
}

// the fold path's group pairs: n x partial blocks x groups x {sum, sumsq}
static size_t gn_fold_ws_bytes(int n, int c, int hw, int groups) {
    return (size_t)n * gn_blocks(n, c, hw, tuning().gn_fold_cap) * groups * 2 * sizeof(float);
}

extern "C" size_t c2d_groupnorm_run_workspace_size(int n, int c, int hw, int groups) {
    if (n <= 0 || c <= 0 || hw <= 0 || groups <= 0 || c % groups) return 0;
    if (gn_use_fused(n, c, hw, groups)) return 0;
    const size_t multi = c2d_groupnorm_workspace_size(n, c, hw) + (size_t)n * c * 2 * sizeof(float);
    const size_t fold = gn_fold_ws_bytes(n, c, hw, groups);
    return fold > multi ? fold : multi;
}

extern "C" int c2d_groupnorm(const void* src0, const void* src1, int c0, int c1, int n, int hw, int groups, float eps,
                             const float* gamma, const float* beta, int silu, void* out, void* ws, size_t ws_bytes,
                             void* stream) {
    if (!src0 || !gamma || !beta || !out) return C2D_E_ARG;
    if (c1 > 0 && !src1) return C2D_E_ARG;
    const int cin = c0 + c1;
    if ((c0 & 7) || (c1 & 7) || cin <= 0 || groups <= 0 || cin % groups) return C2D_E_SHAPE;
    if (cin / groups > 256 || n <= 0 || hw <= 0) return C2D_E_SHAPE;
    if (!aligned16(src0) || (src1 && !aligned16(src1)) || !aligned16(out)) return C2D_E_ALIGN;
    hipStream_t s = (hipStream_t)stream;
    if (gn_use_fused(n, cin, hw, groups)) {
        const int cb = gn_fused_cb(n, cin, groups);
        hipLaunchKernelGGL(gn_fused_kernel<256>, dim3((cin + cb - 1) / cb, n), dim3(256), 0, s, (const f16*)src0,
                           (const f16*)src1, c0, c1, hw, cin / groups, cb, eps, gamma, beta, silu, (f16*)out);
        return check_launch();
    }
    if (!ws || ws_bytes < c2d_groupnorm_run_workspace_size(n, cin, hw, groups) || !aligned16(ws)) return C2D_E_ARG;
    if (gn_use_fold(n, cin, hw, groups))   // ws sized for the group pairs too (gn_fold_ws_bytes)
        return gn_fold_run(src0, src1, c0, c1, n, hw, 0, groups, eps, gamma, beta, silu, out, ws, s);
    const size_t part = c2d_groupnorm_workspace_size(n, cin, hw);
    float* scale = reinterpret_cast<float*>(static_cast<char*>(ws) + part);
    float* shift = scale + (size_t)n * cin;
    int rc = c2d_groupnorm_stats(src0, src1, c0, c1, n, hw, groups, eps, gamma, beta, scale, shift, ws, stream);
    if (rc != C2D_OK) return rc;
    return c2d_groupnorm_apply(src0, src1, c0, c1, n, hw, scale, shift, silu, out, stream);
}

extern "C" size_t c2d_groupnorm_pad_workspace_size(int n, int c, int h, int w) {
    if (n <= 0 || c <= 0 || h <= 0 || w <= 0) return 0;
    const size_t multi = c2d_groupnorm_workspace_size(n, c, h * w) + (size_t)n * c * 2 * sizeof(float);
    const size_t fold = gn_fold_ws_bytes(n, c, h * w, c < 256 ? c : 256);   // the most groups the fold takes
    return fold > multi ? fold : multi;
}

extern "C" int c2d_groupnorm_pad(const void* src0, const void* src1, int c0, int c1, int n, int h, int w, int groups,
                                 float eps, const float* gamma, const float* beta, int silu, void* out, void* ws,
                                 size_t ws_bytes, void* stream) {
    if (!src0 || !gamma || !beta || !out || !ws) return C2D_E_ARG;
    if (c1 > 0 && !src1) return C2D_E_ARG;
    const int cin = c0 + c1;
    if ((c0 & 7) || (c1 & 7) || cin <= 0 || groups <= 0 || cin % groups) return C2D_E_SHAPE;
    if (cin / groups > 256 || n <= 0 || h <= 0 || w <= 0 || (cin >> 3) > 512) return C2D_E_SHAPE;
    if (!aligned16(src0) || (src1 && !aligned16(src1)) || !aligned16(out) || !aligned16(ws)) return C2D_E_ALIGN;
    const int hw = h * w;
    if (ws_bytes < c2d_groupnorm_pad_workspace_size(n, cin, h, w)) return C2D_E_ARG;
    if (gn_use_fold(n, cin, hw, groups))
        return gn_fold_run(src0, src1, c0, c1, n, hw, w + 2, groups, eps, gamma, beta, silu, out, ws,
                           (hipStream_t)stream);
    const size_t part = c2d_groupnorm_workspace_size(n, cin, hw);
    float* scale = reinterpret_cast<float*>(static_cast<char*>(ws) + part);
    float* shift = scale + (size_t)n * cin;
    int rc = c2d_groupnorm_stats(src0, src1, c0, c1, n, hw, groups, eps, gamma, beta, scale, shift, ws, stream);
    if (rc != C2D_OK) return rc;
    const int nch = cin >> 3;
    const int L = nch < 256 ? nch : 256, R = 256 / L;
    const int npix = (h + 2) * (w + 2);
    int bx = (gn_apply_blocks() + n - 1) / n;
    const int maxb = (npix + R - 1) / R;
    if (bx > maxb) bx = maxb;
    if (bx < 1) bx = 1;
    if (nch <= 256)
        hipLaunchKernelGGL((gn_apply_kernel<1, true>), dim3(bx, n), dim3(256), 0, (hipStream_t)stream, (const f16*)src0,
                           (const f16*)src1, c0, c1, hw, scale, shift, silu, (f16*)out, w + 2);
    else
        hipLaunchKernelGGL((gn_apply_kernel<2, true>), dim3(bx, n), dim3(256), 0, (hipStream_t)stream, (const f16*)src0,
                           (const f16*)src1, c0, c1, hw, scale, shift, silu, (f16*)out, w + 2);
    return check_launch();
}
