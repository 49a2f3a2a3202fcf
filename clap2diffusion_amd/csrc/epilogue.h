// Shared GEMM epilogue body for the implicit-GEMM kernels (included by igemm.hip
// after IgemmParams).  The MFMA kernels first write their fp32 accumulators as
// a row-major image into the (now free) LDS staging ring; epi_rows then applies
//   out[m, j] = act(acc + bias[j]) + temb[n(m), j] + resid[m, j]
//   (GEGLU: (h + bh) * gelu(g + bg) [+ resid], packed [16 h | 16 g] per 32 rows)
// in one compact loop over 16-B output chunks: coalesced 16-B loads / stores,
// one fp16 rounding at the end, and a few hundred instructions of code instead
// of a fully unrolled per-register epilogue (which ran to ~50k instructions with
// the runtime activation branches and thrashed the instruction cache).
#pragma once

namespace c2d {

// W-column chunk body (W = 8: 16-B loads / stores; W = 4: 8-B, for outputs whose
// width, leading dimensions or base addresses are only 4-element aligned, e.g. the
// 4-channel conv_out).  img: fp32 [ROWS][pitchf] image of the block's rows m0..
// and packed weight columns jp0 .. jp0 + COLS (COLS % 8 == 0; GEGLU: % 32 == 0).
// The image geometry and the GEGLU flag are template parameters so the chunk ->
// (row, column) split is constant-divisor arithmetic: with run-time divisors the
// integer divisions cost as much VALU per chunk as the GELU itself.
template <int W, bool GG, int ROWS, int COLS>
__device__ __forceinline__ void epi_rows_t(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                           int lane) {
    typedef _Float16 hv __attribute__((ext_vector_type(W)));
    constexpr int CPR = GG ? COLS / (2 * W) : COLS / W;   // W-wide output chunks per row
    constexpr int CPT = 16 / W;                           // GEGLU: chunks per 32-row tile
    static_assert(COLS % (GG ? 32 : 8) == 0, "epilogue image width");
    const int hw = p.oh * p.ow;
    const int out_cols = GG ? (p.cout >> 1) : p.cout;
    // image of all ROWS rows when they cannot straddle one (m0 is a multiple of ROWS)
    const int n_all = (hw % ROWS) == 0 ? m0 / hw : -1;
#pragma unroll 2
    for (int c = lane; c < ROWS * CPR; c += 64) {
        const int row = c / CPR, cc = c - row * CPR;
        const int m = m0 + row;
        int sc, jp, j;                                       // image column, packed row, output column
        if constexpr (GG) {
            const int t = cc / CPT, q = cc - t * CPT;
            sc = t * 32 + q * W;
            jp = jp0 + sc;
            j = ((jp0 + t * 32) >> 1) + q * W;
        } else {
            sc = cc * W;
            jp = jp0 + sc;
            j = jp;
        }
        if (m >= p.M || j >= out_cols) continue;
        const float* src = img + row * pitchf + sc;
        float v[W];
#pragma unroll
        for (int r = 0; r < W; r += 4) {
            const float4 x = *reinterpret_cast<const float4*>(src + r);
            v[r] = x.x; v[r + 1] = x.y; v[r + 2] = x.z; v[r + 3] = x.w;
        }
        if (p.bias) {
#pragma unroll
            for (int r = 0; r < W; r += 4) {
                const float4 bb = *reinterpret_cast<const float4*>(p.bias + jp + r);
                v[r] += bb.x; v[r + 1] += bb.y; v[r + 2] += bb.z; v[r + 3] += bb.w;
            }
        }
        if constexpr (GG) {
            float g[W];
#pragma unroll
            for (int r = 0; r < W; r += 4) {
                const float4 x = *reinterpret_cast<const float4*>(src + 16 + r);
                g[r] = x.x; g[r + 1] = x.y; g[r + 2] = x.z; g[r + 3] = x.w;
                if (p.bias) {
                    const float4 bb = *reinterpret_cast<const float4*>(p.bias + jp + 16 + r);
                    g[r] += bb.x; g[r + 1] += bb.y; g[r + 2] += bb.z; g[r + 3] += bb.w;
                }
            }
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] *= gelu_f(g[r]);
        } else if (p.act == C2D_ACT_GELU) {
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] = gelu_f(v[r]);
        } else if (p.act == C2D_ACT_RELU) {
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] = fmaxf(v[r], 0.f);
        } else if (p.act == C2D_ACT_SILU) {
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] = silu_f(v[r]);
        } else if (p.act == C2D_ACT_QUICK_GELU) {   // CLIP's quick_gelu x * sigmoid(1.702 x)
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] = sigmoid_lin(v[r], 1.702f);
        }
        if (p.temb) {
            const hv tt = *reinterpret_cast<const hv*>(p.temb + (size_t)(n_all >= 0 ? n_all : m / hw) * p.temb_ld + j);
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] += (float)tt[r];
        }
        if (p.resid) {
            const hv rr = *reinterpret_cast<const hv*>(p.resid + (size_t)m * p.resid_ld + j);
#pragma unroll
            for (int r = 0; r < W; ++r) v[r] += (float)rr[r];
        }
        hv o;
#pragma unroll
        for (int r = 0; r < W; ++r) o[r] = (f16)v[r];
        *reinterpret_cast<hv*>(p.out + (size_t)m * p.out_ld + j) = o;
    }
}

// ROWS x COLS fp32 image -> outputs; picks the 16-B (W = 8) form when the output
// width, the leading dimensions and the base addresses allow it
template <int ROWS, int COLS>
__device__ __forceinline__ void epi_rows(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                         int lane) {
    const bool gg = p.act == C2D_ACT_GEGLU;
    const int out_cols = gg ? (p.cout >> 1) : p.cout;
    const uintptr_t al = (uintptr_t)p.out | (uintptr_t)p.resid | (uintptr_t)p.temb;
    const bool wide = ((out_cols | p.out_ld | (p.resid ? p.resid_ld : 0) | (p.temb ? p.temb_ld : 0)) & 7) == 0 &&
                      (al & 15) == 0;
    if constexpr (COLS % 32 == 0) {
        if (gg) {
            if (wide) epi_rows_t<8, true, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
            else epi_rows_t<4, true, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
            return;
        }
    }
    if (wide) epi_rows_t<8, false, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
    else epi_rows_t<4, false, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
}

}  // namespace c2d
