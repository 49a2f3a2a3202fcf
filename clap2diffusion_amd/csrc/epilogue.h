// Shared GEMM epilogue body for the implicit-GEMM kernels (included by igemm.hip
// after IgemmParams).  After the main loop a kernel stages its fp32 accumulators,
// bias already added, as a row-major image in the (now free) LDS ring, one pass of
// up to 32 rows per wave at a time; epi_pass then applies
//   out[m, j] = act(img[m, j]) + temb[n(m), j] + resid[m, j]
//   (GEGLU: img_h * gelu(img_g) [+ resid], packed [16 h | 16 g] per 32 rows)
// over 16-B output chunks: coalesced 16-B loads / stores, one fp16 rounding.
//
// Latency.  The residual / temb chunks of a pass are loaded (unconditionally:
// out-of-range rows and columns clamped to a valid address, only the store is
// predicated) BEFORE the kernel writes the pass's image, so their HBM latency runs
// under the image write and the pass waits once.  The bias rides the image write
// (loaded once per tile in the accumulator layout).  The earlier form branched on
// each optional operand around its load and its use inside the chunk loop, so every
// chunk paid up to three serialised global round trips (an s_waitcnt vmcnt(0) after
// each load): +8-10 us per launch for a residual on a one-round 256 x 320 tile grid.
#pragma once

namespace c2d {

// RES / TEMB: 1 / 0 = the operand is / is not there (fast forms, unconditional loads);
// -1 = decided at run time from p.resid / p.temb (the generic form: 4-wide outputs and
// GEGLU with a residual, which the UNet never issues -- kept correct, not fast)
// NT: threads sharing the image (64: a wave's own image; 512: a workgroup image).
// RG: 0 = image row r is output row m0 + r; else the image holds groups of 32 rows whose
// output rows lie RG apart (m0 + (r / 32) RG + r % 32: the row groups of a 2-row-group tile).
// WB: also write each stored value (as rounded to fp16) back over its image entry, so that a pass
// over the image afterwards sees exactly the output (epi_pass_wb: the producer-side GroupNorm moments)
template <int W, bool GG, int ROWS, int COLS, int RES, int TEMB, int NT = 64, int RG = 0, bool WB = false>
struct EpiPass {
    typedef _Float16 hv __attribute__((ext_vector_type(W)));
    static constexpr int CPR = GG ? COLS / (2 * W) : COLS / W;   // W-wide output chunks per row
    static constexpr int CPT = 16 / W;                           // GEGLU: chunks per 32-row tile
    static constexpr int NCH = ROWS * CPR;
    static constexpr int NIT = (NCH + NT - 1) / NT;
    static_assert(COLS % (GG ? 32 : 8) == 0, "epilogue image width");
    hv r[RES ? NIT : 1], t[TEMB ? NIT : 1];
    __device__ __forceinline__ static bool has_res(const IgemmParams& p) { return RES > 0 || (RES < 0 && p.resid); }
    __device__ __forceinline__ static bool has_temb(const IgemmParams& p) { return TEMB > 0 || (TEMB < 0 && p.temb); }

    // chunk it of this lane: image row / column, output row / column, store predicate
    __device__ __forceinline__ static void geo(const IgemmParams& p, int m0, int jp0, int lane, int it, int& row,
                                               int& sc, int& m, int& j, bool& ok) {
        int c = lane + NT * it;
        ok = c < NCH;
        c = ok ? c : NCH - 1;
        row = c / CPR;
        const int cc = c - row * CPR;
        if constexpr (GG) {
            const int t = cc / CPT, q = cc - t * CPT;
            sc = t * 32 + q * W;
            j = ((jp0 + t * 32) >> 1) + q * W;
        } else {
            sc = cc * W;
            j = jp0 + sc;
        }
        m = m0 + (RG ? (row >> 5) * RG + (row & 31) : row);
        ok = ok && m < p.M && j < (GG ? (p.cout >> 1) : p.cout);
        if (!ok) { m = m0 < p.M ? m0 : 0; j = 0; }   // a valid address for the unconditional loads
    }

    __device__ __forceinline__ void prefetch(const IgemmParams& p, int m0, int jp0, int lane) {
        if constexpr (RES != 0 || TEMB != 0) {
            const int hw = p.oh * p.ow;
            const int n_all = (RG == 0 && (hw % ROWS) == 0) ? m0 / hw : -1;   // all ROWS rows in one image
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                int row, sc, m, j;
                bool ok;
                geo(p, m0, jp0, lane, it, row, sc, m, j, ok);
                if (TEMB != 0 && has_temb(p))
                    t[it] = *reinterpret_cast<const hv*>(p.temb + (size_t)(ok ? (n_all >= 0 ? n_all : m / hw) : 0) *
                                                                      p.temb_ld + j);
                if (RES != 0 && has_res(p)) r[it] = *reinterpret_cast<const hv*>(p.resid + (size_t)m * p.resid_ld + j);
            }
        }
    }

    // one chunk: act(image) [+ temb] [+ residual] -> fp16 -> store (predicated)
    __device__ __forceinline__ static void body(const IgemmParams& p, const float* img, int pitchf, int row, int sc,
                                                int m, int j, bool ok, const hv& rr, const hv& tt) {
        const float* src = img + row * pitchf + sc;
        float v[W];
#pragma unroll
        for (int q = 0; q < W; q += 4) {
            const float4 x = *reinterpret_cast<const float4*>(src + q);
            v[q] = x.x; v[q + 1] = x.y; v[q + 2] = x.z; v[q + 3] = x.w;
        }
        if constexpr (GG) {
#pragma unroll
            for (int q = 0; q < W; q += 4) {
                const float4 y = *reinterpret_cast<const float4*>(src + 16 + q);
                v[q] *= gelu_sig(y.x); v[q + 1] *= gelu_sig(y.y); v[q + 2] *= gelu_sig(y.z); v[q + 3] *= gelu_sig(y.w);
            }
        } else if (p.act == C2D_ACT_GELU) {
#pragma unroll
            for (int q = 0; q < W; ++q) v[q] = gelu_f(v[q]);
        } else if (p.act == C2D_ACT_RELU) {
#pragma unroll
            for (int q = 0; q < W; ++q) v[q] = fmaxf(v[q], 0.f);
        } else if (p.act == C2D_ACT_SILU) {
#pragma unroll
            for (int q = 0; q < W; ++q) v[q] = silu_f(v[q]);
        } else if (p.act == C2D_ACT_QUICK_GELU) {   // CLIP's quick_gelu x * sigmoid(1.702 x)
#pragma unroll
            for (int q = 0; q < W; ++q) v[q] = sigmoid_lin(v[q], 1.702f);
        }
        if (TEMB != 0 && has_temb(p)) {
#pragma unroll
            for (int q = 0; q < W; ++q) v[q] += (float)tt[q];
        }
        if (RES != 0 && has_res(p)) {
#pragma unroll
            for (int q = 0; q < W; ++q) v[q] += (float)rr[q];
        }
        hv o;
#pragma unroll
        for (int q = 0; q < W; ++q) o[q] = (f16)v[q];
        if (ok) *reinterpret_cast<hv*>(p.out + (size_t)m * p.out_ld + j) = o;
        if constexpr (WB) {
            float* dst = const_cast<float*>(src);
#pragma unroll
            for (int q = 0; q < W; q += 4)
                *reinterpret_cast<float4*>(dst + q) = make_float4((float)o[q], (float)o[q + 1], (float)o[q + 2], (float)o[q + 3]);
        }
    }

    __device__ __forceinline__ void finish(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                           int lane) const {
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            int row, sc, m, j;
            bool ok;
            geo(p, m0, jp0, lane, it, row, sc, m, j, ok);
            body(p, img, pitchf, row, sc, m, j, ok, r[RES ? it : 0], t[TEMB ? it : 0]);
        }
    }

    // compact form: one rolled loop, the chunk's residual / temb loads issued together
    // with its image read (one wait per chunk, two chunks per trip); for kernels whose
    // epilogue code runs from a cold instruction cache once per tile (the unrolled
    // prefetch form grew their code past the short-branch range and ran slower)
    __device__ __forceinline__ static void compact(const IgemmParams& p, const float* img, int pitchf, int m0,
                                                   int jp0, int lane) {
        const int hw = p.oh * p.ow;
        const int n_all = (RG == 0 && (hw % ROWS) == 0) ? m0 / hw : -1;
#pragma unroll 2
        for (int it = 0; it < NIT; ++it) {
            int row, sc, m, j;
            bool ok;
            geo(p, m0, jp0, lane, it, row, sc, m, j, ok);
            hv rr, tt;
            if (TEMB != 0 && has_temb(p))
                tt = *reinterpret_cast<const hv*>(p.temb + (size_t)(ok ? (n_all >= 0 ? n_all : m / hw) : 0) * p.temb_ld + j);
            if (RES != 0 && has_res(p)) rr = *reinterpret_cast<const hv*>(p.resid + (size_t)m * p.resid_ld + j);
            body(p, img, pitchf, row, sc, m, j, ok, rr, tt);
        }
    }
};

// one pass: prefetch the pass's residual / temb, let the kernel write the image
// (write_img(): bias-added accumulators -> LDS, this wave's rows only), wait for the
// LDS writes, finish.  The wave reads back only its own image, so a wave barrier suffices.
template <bool COMPACT, int NT, int RG, int W, bool GG, int ROWS, int COLS, int RES, int TEMB, class WriteImg>
__device__ __forceinline__ void epi_pass_t(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                           int lane, WriteImg&& write_img) {
    typedef EpiPass<W, GG, ROWS, COLS, RES, TEMB, NT, RG> EP;
    auto sync = [&]() __attribute__((always_inline)) {
        if constexpr (NT == 64) {   // a wave's own image
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
        } else {
            // LDS-only workgroup barrier: __syncthreads' release fence would also wait for
            // the previous pass's global stores (vmcnt(0)) and serialise their drain
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
            asm volatile("" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
    };
    if constexpr (COMPACT) {
        write_img();
        sync();   // image written
        EP::compact(p, img, pitchf, m0, jp0, lane);
    } else {
        EP ep;
        ep.prefetch(p, m0, jp0, lane);
        write_img();
        sync();
        ep.finish(p, img, pitchf, m0, jp0, lane);
    }
    sync();       // image reads done before the next pass rewrites it
}

// One compact workgroup pass (16-B outputs, no GEGLU: the caller checked) that leaves the stored
// values in the image and runs after() over it before the next pass may rewrite it
template <int NT, int RG, int ROWS, int COLS, class WriteImg, class After>
__device__ __forceinline__ void epi_pass_wb(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                            int lane, WriteImg&& write_img, After&& after) {
    typedef EpiPass<8, false, ROWS, COLS, -1, -1, NT, RG, true> EP;
    auto sync = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    write_img();
    sync();
    EP::compact(p, img, pitchf, m0, jp0, lane);
    sync();
    after();
    sync();
}

// GroupNorm moments of a BM x BN output tile (IgemmParams::gn_mom) from its workgroup-image epilogue: NPASS
// epi_pass_wb passes of ROWS image rows (image row r = output row m0 + 16 * 2 pass + (r / 32) RG + r % 32),
// write_img(pass) writing pass's bias-added accumulators.  Each pass leaves its stored fp16 values in the
// image; thread c < BN then adds column n0 + c's values, shifted by the tile's first one, over the pass's rows.
// At the end: per column (mean, M2) over the BM rows -> LDS -> per group (fixed channel order, equal counts)
// -> {mean, M2} of (image, tile, group).  Needs BM-row tiles inside one image, BN % cpg == 0, n0 % cpg == 0.
template <int NPASS, int ROWS, int BN, int BM, int RG, class WriteImg>
__device__ __forceinline__ void epi_gn_moments(const IgemmParams& p, float* img, int pitchb, int m0, int n0, int tid,
                                               WriteImg&& write_img) {
    float sh = 0.f, s1 = 0.f, s2 = 0.f;
    static_for<0, NPASS>([&](auto pass) __attribute__((always_inline)) {
        constexpr int b0 = 2 * decltype(pass)::value;
        epi_pass_wb<512, RG, ROWS, BN>(p, img, pitchb, m0 + b0 * 16, n0, tid,
                                       [&]() __attribute__((always_inline)) { write_img(pass); },
                                       [&]() __attribute__((always_inline)) {
            if (tid < BN) {
                if constexpr (b0 == 0) sh = img[tid];
#pragma unroll 8
                for (int r = 0; r < ROWS; ++r) {
                    const float d = img[r * pitchb + tid] - sh;
                    s1 += d;
                    s2 = fmaf(d, d, s2);
                }
            }
        });
    });
    float2* chm = reinterpret_cast<float2*>(img);   // the image is free again (epi_pass_wb's last barrier)
    if (tid < BN) chm[tid] = make_float2(sh + s1 * (1.0f / BM), s2 - s1 * s1 * (1.0f / BM));
    __syncthreads();
    const int cpg = p.gn_cpg, ng = BN / cpg;
    if (tid < ng) {
        float mg = 0.f;
        for (int i = 0; i < cpg; ++i) mg += chm[tid * cpg + i].x;
        mg /= (float)cpg;
        float q = 0.f;
        for (int i = 0; i < cpg; ++i) {
            const float2 e = chm[tid * cpg + i];
            const float d = e.x - mg;
            q += e.y + (float)BM * d * d;
        }
        const int hw = p.oh * p.ow, nimg = m0 / hw, tpi = hw / BM, groups = p.cout / cpg;
        const size_t slot = ((size_t)nimg * tpi + (m0 - nimg * hw) / BM) * groups + n0 / cpg + tid;
        reinterpret_cast<float2*>(p.gn_mom)[slot] = make_float2(mg, q);
    }
}

// ROWS x COLS image pass -> outputs; picks the 16-B (W = 8) form when the output
// width, the leading dimensions and the base addresses allow it
template <int ROWS, int COLS, bool COMPACT, int NT = 64, int RG = 0, class WriteImg>
__device__ __forceinline__ void epi_pass(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                         int lane, WriteImg&& w) {
    const bool gg = p.act == C2D_ACT_GEGLU;
    const int out_cols = gg ? (p.cout >> 1) : p.cout;
    const uintptr_t al = (uintptr_t)p.out | (uintptr_t)p.resid | (uintptr_t)p.temb;
    const bool wide = ((out_cols | p.out_ld | (p.resid ? p.resid_ld : 0) | (p.temb ? p.temb_ld : 0)) & 7) == 0 &&
                      (al & 15) == 0;
    if constexpr (COMPACT) {   // operands decided at run time: one body per width
        if constexpr (COLS % 32 == 0) {
            if (gg) {
                if (wide) epi_pass_t<true, NT, RG, 8, true, ROWS, COLS, -1, 0>(p, img, pitchf, m0, jp0, lane, w);
                else epi_pass_t<true, NT, RG, 4, true, ROWS, COLS, -1, 0>(p, img, pitchf, m0, jp0, lane, w);
                return;
            }
        }
        if (wide) epi_pass_t<true, NT, RG, 8, false, ROWS, COLS, -1, -1>(p, img, pitchf, m0, jp0, lane, w);
        else epi_pass_t<true, NT, RG, 4, false, ROWS, COLS, -1, -1>(p, img, pitchf, m0, jp0, lane, w);
        return;
    }
    if constexpr (COLS % 32 == 0) {
        if (gg) {   // GEGLU never carries a time embedding (c2d_conv2d_igemm validation)
            if (wide && !p.resid) epi_pass_t<COMPACT, NT, RG, 8, true, ROWS, COLS, 0, 0>(p, img, pitchf, m0, jp0, lane, w);
            else epi_pass_t<COMPACT, NT, RG, 4, true, ROWS, COLS, -1, 0>(p, img, pitchf, m0, jp0, lane, w);
            return;
        }
    }
    if (!wide) epi_pass_t<COMPACT, NT, RG, 4, false, ROWS, COLS, -1, -1>(p, img, pitchf, m0, jp0, lane, w);
    else if (p.resid) {
        if (p.temb) epi_pass_t<COMPACT, NT, RG, 8, false, ROWS, COLS, 1, 1>(p, img, pitchf, m0, jp0, lane, w);
        else epi_pass_t<COMPACT, NT, RG, 8, false, ROWS, COLS, 1, 0>(p, img, pitchf, m0, jp0, lane, w);
    } else {
        if (p.temb) epi_pass_t<COMPACT, NT, RG, 8, false, ROWS, COLS, 0, 1>(p, img, pitchf, m0, jp0, lane, w);
        else epi_pass_t<COMPACT, NT, RG, 8, false, ROWS, COLS, 0, 0>(p, img, pitchf, m0, jp0, lane, w);
    }
}

// bias of the 4 consecutive packed columns j .. j + 3 (zeros without a bias / past cout;
// cout % 4 == 0, so a run is either wholly inside or wholly past)
__device__ __forceinline__ f32x4 bias4(const IgemmParams& p, int j) {
    if (!p.bias || j >= p.cout) return (f32x4){0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const f32x4*>(p.bias + j);
}

// ---------------------------------------------------------------------------
// Plain form (outputs without a residual or a time embedding: QKV, to_q, GEGLU,
// proj_in): the round-1 loop, bias read per chunk from p.bias, the image holding the
// raw accumulators.  Measured faster than the hoisted / workgroup forms on these
// multi-round tile grids (L0 QKV 63.6 vs 71.5 us, L0 GEGLU 188.8 vs 203.3 us on tile 40).
// W-column chunk body (W = 8: 16-B loads / stores; W = 4: 8-B, for outputs whose
// width, leading dimensions or base addresses are only 4-element aligned, e.g. the
// 4-channel conv_out).  img: fp32 [ROWS][pitchf] image of the block's rows m0..
// and packed weight columns jp0 .. jp0 + COLS (COLS % 8 == 0; GEGLU: % 32 == 0).
// The image geometry and the GEGLU flag are template parameters so the chunk ->
// (row, column) split is constant-divisor arithmetic: with run-time divisors the
// integer divisions cost as much VALU per chunk as the GELU itself.
template <int W, bool GG, int ROWS, int COLS>
__device__ __forceinline__ void epi_rows_plain_t(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
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
            for (int r = 0; r < W; ++r) v[r] *= gelu_sig(g[r]);
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
__device__ __forceinline__ void epi_rows_plain(const IgemmParams& p, const float* img, int pitchf, int m0, int jp0,
                                         int lane) {
    const bool gg = p.act == C2D_ACT_GEGLU;
    const int out_cols = gg ? (p.cout >> 1) : p.cout;
    const uintptr_t al = (uintptr_t)p.out | (uintptr_t)p.resid | (uintptr_t)p.temb;
    const bool wide = ((out_cols | p.out_ld | (p.resid ? p.resid_ld : 0) | (p.temb ? p.temb_ld : 0)) & 7) == 0 &&
                      (al & 15) == 0;
    if constexpr (COLS % 32 == 0) {
        if (gg) {
            if (wide) epi_rows_plain_t<8, true, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
            else epi_rows_plain_t<4, true, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
            return;
        }
    }
    if (wide) epi_rows_plain_t<8, false, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
    else epi_rows_plain_t<4, false, ROWS, COLS>(p, img, pitchf, m0, jp0, lane);
}

}  // namespace c2d
