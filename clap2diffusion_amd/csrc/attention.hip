// Flash-style attention forward for gfx950 (MFMA f32_16x16x32_f16) and the
// HTSAT Swin window attention.
//
// attention_fwd: one workgroup = 4 waves = 128 queries of one (batch, head);
// each wave owns 32 queries (two 16-query groups).  Key/value tiles of 64 keys
// are register-staged into LDS (K rows padded to an odd number of 16-B slots,
// V rows padded for conflict-free ds_read_b64_tr_b16).  Scores are computed
// transposed, S^T = K Q^T, so each lane holds 16 keys of ONE query: the softmax
// row max needs two lane shuffles, the row sum none until the end, and the
// exponentiated P fragment is already the B operand of O^T = V^T P^T (the k
// order of the PV product is permuted to match, V^T comes from the transposed
// LDS read).  O^T accumulators keep the query on the lane, so the online-softmax
// rescale is lane-local.  Softmax in fp32 with exp2 and a folded log2(e) scale.
#include "common.h"
#include <stdlib.h>

namespace c2d {

#ifndef ATTN_WPE
#define ATTN_WPE 4
#endif

#ifndef C2D_TUNE_ATTN_BUFLD
#define C2D_TUNE_ATTN_BUFLD 1   // whole key tiles staged by buffer loads off a per-tile SGPR base (round 6); 0 = A/B builds
#endif

#ifndef C2D_TUNE_ATTN_PRIO
#define C2D_TUNE_ATTN_PRIO 0
#endif
#ifndef C2D_TUNE_ATTN_W8_MIN
// d = 40: the 8-wave (256-query) blocks only when the grid has at least this many of them (one per CU); a
// smaller grid runs 4-wave blocks, twice as many (round 6, scripts/bench_attn.py, same box: c2's CFG-shared
// first self-attention, 8 heads x 16 blocks, 69.6 / 68.2 -> 53.4 / 55.4 us; at 256 blocks, c2's 16 heads,
// the 8-wave form stays ahead, 77.9 vs 80.9 us); 0 = always 8-wave (A/B builds)
#define C2D_TUNE_ATTN_W8_MIN 256
#endif

#ifndef C2D_TUNE_ATTN80
#define C2D_TUNE_ATTN80 1   // d = 80: 1 = the PV row-sum column (round 6), 0 = VALU row sums (round 5; A/B builds)
#endif

template <int D> struct AttnCfg {
    // K dim of QK^T: full 32-deep chunks on 16x16x32 MFMAs plus, when the rest is
    // exactly 16 deep (d = 80), one 16x16x16 MFMA into a separate accumulator
    // (added with VALU) instead of a zero-padded 32 chunk.  Round 6 chained it into the
    // 32-deep accumulators instead (same C/D layout; 3 % faster at L1): the resident-K/V
    // 64-key case (test_attention[3-8-300-64-80]) came out wrong (rel-L2 0.14), so no
    // mixed-shape MFMA accumulation chain
    // d < 64 and not a multiple of 32 (d = 40): the whole QK^T on 16x16x16 MFMAs
    // over 16-deep chunks (K = 48 instead of a zero-padded 64)
    static constexpr bool C16 = false;   // measured slower on gfx950: 16x16x16 issues at the 16x16x32 cycle count
    static constexpr int NC16 = C16 ? (D + 15) / 16 : 0;
    static constexpr int NDC = D / 32;
    static constexpr bool TAIL = !C16 && (D % 32) == 16;
    static constexpr int DP = C16 ? NC16 * 16 : TAIL ? NDC * 32 + 16 : (D + 31) / 32 * 32;
    static constexpr int NDC_FULL = C16 ? 0 : TAIL ? NDC : DP / 32;  // 32-deep chunks actually issued
    // N dim of PV, multiple of 16.  d = 80: one more 16-column tile (96) so the PV MFMAs also carry the
    // row sum (SUM_MFMA): 4 more MFMAs per wave-tile against 32 VALU adds of the per-lane sums
    static constexpr int DV = (D == 80 && C2D_TUNE_ATTN80) ? 96 : (D + 15) / 16 * 16;
    static constexpr int NDT = DV / 16;
    // K rows: 128-B rows with the 16-B chunk XOR swizzle (chunk ^ ((row >> 1) & 7)) when
    // DP = 64 (conflict-free QK^T fragment reads, PMC-verified need: the padded
    // 144-B rows measured 2-way conflicts); otherwise rows padded to an odd number of slots
    static constexpr bool KSW = DP == 64;
    static constexpr int KS = KSW ? 128 : DP * 2 + 16;
    static constexpr int VS = (DV == 48) ? 96 : (DV == 64 || DV == 80) ? 160 : (DV == 160) ? 352 : DV * 2 + 32;
    static constexpr int DCH = D / 8;                  // real 16-B chunks per row
    static constexpr int NLD = (64 * DCH + 255) / 256; // staged chunks per thread per tile
    static constexpr int K_BYTES = 64 * KS;
    static constexpr int V_BYTES = 64 * VS;
    static constexpr bool SUM_MFMA = DV > D;           // a spare V column carries the row sum
};

// Row max of a lane's 16 scores and its 3 partner lanes (l ^ 16, l ^ 32): two gfx950
// lane-swap VALU ops instead of two ds_bpermute LDS round trips.  The file is built with
// -fno-honor-nans (build.py): IEEE-mode fmaxf would prefix every MFMA-output operand with a
// canonicalising v_max; without it the chain folds into v_max3 (inline asm v_max3 made the
// compiler pad every asm statement with s_nop instead).
__device__ __forceinline__ float lane_max16(const f32x4 (&s)[4]) {
    float m = s[0][0];
#pragma unroll
    for (int kg = 0; kg < 4; ++kg)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, s[kg][r]);
    return m;
}
__device__ __forceinline__ float quad_max(float m) {   // max over lanes l, l ^ 16, l ^ 32, l ^ 48
    const unsigned u = __float_as_uint(m);
    const auto x32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);   // {own, l ^ 32} per lane
    const float m2 = fmaxf(__uint_as_float(x32[0]), __uint_as_float(x32[1]));
    const unsigned u2 = __float_as_uint(m2);
    const auto x16 = __builtin_amdgcn_permlane16_swap(u2, u2, false, false); // {own, l ^ 16} per lane
    return fmaxf(__uint_as_float(x16[0]), __uint_as_float(x16[1]));
}

template <int D>
__device__ __forceinline__ int k_off(int row, int ch) {   // byte offset of 16-B chunk ch of K row
    using C = AttnCfg<D>;
    return C::KSW ? row * 128 + ((ch ^ ((row >> 1) & 7)) << 4) : row * C::KS + ch * 16;
}

// NEGC: Q is pre-scaled by scale*log2(e) when its fragments load and every S^T tile
// starts its MFMA chain from C = -m_run (a per-query register block, rewritten only
// when the running max moves), so the MFMA emits s*scale*log2e - m directly and the
// softmax is exp2 alone: one v_fma per score less on the VALU issue that bounds the
// d = 40 kernel.  m_run starts at 0 and the first tile always rebases it to the tile max.
// d <= 64: held to 128 VGPRs = 4 waves per SIMD (from 140 = 3); the compiler parks two
// 8-B values in scratch (one L1-resident reload pair per key tile).  d = 80 / 160 would
// spill hundreds of bytes at that bound, so they keep the free allocation.
// RES (lk <= 128, the 77-key cross-attention): every key tile stays resident in LDS
// (one slot per tile, staged once) and the workgroup walks `qpb` consecutive 128-query
// blocks of its (image, head) over them -- the streaming form re-staged K/V and paid
// the staging latency once per 128 queries for ~6 MFLOP of work.
// KBIAS: an additive score bias (attention_mask of the processor API: fp32
// kbias[b * kb_ldb + h * kb_ldh + query * kb_ldq + key], natural-log units, added to
// q.k * scale before the softmax); only with NEGC = false.  The scores move to the log2
// domain as they are biased (s = q.k * scale * log2 e + bias * log2 e, kb_mul = log2 e), so
// no bias is ever multiplied by 1 / scale: a finite bias stays finite (finfo.min * log2 e
// is clamped to -FLT_MAX, so a row of finfo.min entries is a row of equal scores -> the
// uniform average of V, as torch gives), -inf stays -inf.  With a bias, the running max
// starts at -inf, padded keys are -inf (never 1e30-style finite values that could win a
// row whose real keys are all -inf / finfo.min), exp2 uses 0 for a row max still at -inf
// (so an all -inf row has p = 0, l = 0 and comes out NaN, as torch's softmax of it does).
template <int D, bool MASK, bool NEGC, bool RES = false, bool KBIAS = false, int NWV = 4>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(D <= 64 ? ATTN_WPE : 1)))
attn_fwd_kernel(const f16* __restrict__ q, int ldq, const f16* __restrict__ k,
                                                       int ldk, const f16* __restrict__ v, int ldv, f16* __restrict__ o,
                                                       int ldo, int heads, int lq, int lk, float scale_log2,
                                                       int kv_div, int nqb, int abl, int qpb = 1,
                                                       const float* __restrict__ kbias = nullptr, int kb_ldb = 0,
                                                       int kb_ldh = 0, float kb_mul = 0.f, int kb_ldq = 0) {
    static_assert(!(KBIAS && NEGC), "key bias only on the fma-softmax form");
    using C = AttnCfg<D>;
    constexpr int NT = 64 * NWV;                              // threads; NWV waves x 32 queries per block
    constexpr int NLD = (64 * C::DCH + NT - 1) / NT;          // staged K / V chunks per thread per tile
    constexpr int SLOT = C::K_BYTES + C::V_BYTES;
    constexpr int NSLOT = RES ? 2 : 1;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Ks = smem;
    char* Vs = smem + C::K_BYTES;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // 8-wave blocks: static priority for the second-dispatched half (waves 4-7), the VALU-issue
    // arbitration loser of each SIMD pair (C2D_TUNE_ATTN_PRIO, A/B)
    if (C2D_TUNE_ATTN_PRIO && NWV == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int qpb_ = RES ? qpb : 1;   // streaming form: one query block (a single-trip loop below)
    const int ngrp = (nqb + qpb_ - 1) / qpb_;
    const int bh = tile / ngrp, qgrp = tile - bh * ngrp;
    const int b = bh / heads, h = bh - b * heads;
    const int bk = b / kv_div;
    const int g = lane >> 4, li = lane & 15;

    // zero the K padding columns once (never rewritten) and the V pad columns
#pragma unroll
    for (int sl = 0; sl < NSLOT; ++sl) {
        for (int idx = tid; idx < 64 * (C::DP / 8 - C::DCH); idx += NT) {
            int row = idx / (C::DP / 8 - C::DCH), ch = C::DCH + idx % (C::DP / 8 - C::DCH);
            *reinterpret_cast<f16x8*>(Ks + sl * SLOT + k_off<D>(row, ch)) = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
        }
        // V pad columns: zeros, except column D = 1.0 when there is one, so the PV
        // product also accumulates the softmax row sum (SUM_MFMA)
        for (int idx = tid; idx < 64 * (C::DV / 8 - C::DCH); idx += NT) {
            int row = idx / (C::DV / 8 - C::DCH), ch = C::DCH + idx % (C::DV / 8 - C::DCH);
            f16x8 z = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
            if (ch == C::DCH) z[0] = (f16)1.0f;
            *reinterpret_cast<f16x8*>(Vs + sl * SLOT + row * C::VS + ch * 16) = z;
        }
    }

    const f16* kbase = k + (size_t)bk * lk * ldk + h * D;
    const f16* vbase = v + (size_t)bk * lk * ldv + h * D;
    f16x8 rk[NLD], rv[NLD];
    // BUFLD (whole key tiles, lk % 64 == 0): the tile's K / V rows through buffer loads whose base is the
    // tile's first row (SGPRs, advanced by SALU per tile) and whose per-lane offsets are loop-invariant,
    // so staging a tile costs no 64-bit address VALU (7 of the d = 40 loop's VALU per wave-tile)
    constexpr bool BUFLD = !MASK && C2D_TUNE_ATTN_BUFLD;
    unsigned koff[NLD], voff[NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int idx = tid + NT * i, row = idx / C::DCH, ch = idx - row * C::DCH;
        koff[i] = (unsigned)(2 * (row * ldk + ch * 8));
        voff[i] = (unsigned)(2 * (row * ldv + ch * 8));
    }
    const char* ukb = uniform_ptr(kbase);
    const char* uvb = uniform_ptr(vbase);
    auto gload = [&](int t) {
        if constexpr (BUFLD) {
            const __amdgpu_buffer_rsrc_t rks = make_rsrc(ukb + (size_t)t * 128 * ldk, (unsigned)(128 * ldk));
            const __amdgpu_buffer_rsrc_t rvs = make_rsrc(uvb + (size_t)t * 128 * ldv, (unsigned)(128 * ldv));
#pragma unroll
            for (int i = 0; i < NLD; ++i) {
                const int idx = tid + NT * i;
                if (NT * i < 64 * C::DCH - (NT - 1) || idx < 64 * C::DCH) {
                    rk[i] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rks, koff[i], 0, 0));
                    rv[i] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rvs, voff[i], 0, 0));
                }
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int idx = tid + NT * i;
            const int row = idx / C::DCH, ch = idx - row * C::DCH;
            // keys past lk re-read the last key: their scores are masked to -inf,
            // so their V rows meet P = 0
            const int key = min(t * 64 + row, lk - 1);
            if (NT * i < 64 * C::DCH - (NT - 1) || idx < 64 * C::DCH) {
                rk[i] = *reinterpret_cast<const f16x8*>(kbase + (size_t)key * ldk + ch * 8);
                rv[i] = *reinterpret_cast<const f16x8*>(vbase + (size_t)key * ldv + ch * 8);
            }
        }
    };
    auto swrite = [&](int sl) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int idx = tid + NT * i;
            if (NT * i < 64 * C::DCH - (NT - 1) || idx < 64 * C::DCH) {
                const int row = idx / C::DCH, ch = idx - row * C::DCH;
                *reinterpret_cast<f16x8*>(Ks + sl * SLOT + k_off<D>(row, ch)) = rk[i];
                *reinterpret_cast<f16x8*>(Vs + sl * SLOT + row * C::VS + ch * 16) = rv[i];
            }
        }
    };

    const int ntiles = (lk + 63) / 64;
    if (RES) {
        gload(0);
        __syncthreads();  // pad zeroing done before the tiles land
        swrite(0);
        if (ntiles > 1) {
            gload(1);
            swrite(1);
        }
        __syncthreads();
    } else {
        gload(0);
        __syncthreads();  // pad zeroing done before the first tile lands
        swrite(0);
        __syncthreads();
    }

    const int qb_end = RES ? min(nqb, (qgrp + 1) * qpb_) : qgrp + 1;
    for (int qb = qgrp * qpb_; qb < qb_end; ++qb) {
    const int q0 = qb * (32 * NWV) + wave * 32;

    // Q fragments (B operand of S^T = K Q^T): query q0 + 16 qg + li, d = 32 dc + 8 g .. +7;
    // tail (16x16x16): d = 32 NDC + 4 g .. +3
    f16x8 qf[2][C::NDC_FULL > 0 ? C::NDC_FULL : 1];
    f16x4 qt[2];
    f16x4 q16[2][C::NC16 > 0 ? C::NC16 : 1];   // C16: d = 16 c + 4 g .. +3
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
        const int qi = q0 + qg * 16 + li;
#pragma unroll
        for (int dc = 0; dc < C::NDC_FULL; ++dc) {
            const int d0 = dc * 32 + g * 8;
            if (qi < lq && d0 < D)
                qf[qg][dc] = *reinterpret_cast<const f16x8*>(q + ((size_t)b * lq + qi) * ldq + h * D + d0);
            else
                qf[qg][dc] = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
        }
#pragma unroll
        for (int c = 0; c < C::NC16; ++c) {
            const int d0 = c * 16 + g * 4;
            q16[qg][c] = (f16x4){0, 0, 0, 0};
            if (qi < lq && d0 < D)
                q16[qg][c] = *reinterpret_cast<const f16x4*>(q + ((size_t)b * lq + qi) * ldq + h * D + d0);
        }
        qt[qg] = (f16x4){0, 0, 0, 0};
        if (C::TAIL) {
            const int d0 = C::NDC * 32 + g * 4;
            if (qi < lq && d0 < D)
                qt[qg] = *reinterpret_cast<const f16x4*>(q + ((size_t)b * lq + qi) * ldq + h * D + d0);
        }
    }

    if (NEGC) {
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) {
#pragma unroll
            for (int dc = 0; dc < C::NDC_FULL; ++dc)
#pragma unroll
                for (int j = 0; j < 8; ++j) qf[qg][dc][j] = (f16)((float)qf[qg][dc][j] * scale_log2);
#pragma unroll
            for (int j = 0; j < 4; ++j) qt[qg][j] = (f16)((float)qt[qg][j] * scale_log2);
        }
    }

    f32x4 acc[C::NDT][2];
#pragma unroll
    for (int dt = 0; dt < C::NDT; ++dt)
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) acc[dt][qg] = (f32x4){0.f, 0.f, 0.f, 0.f};
    constexpr float M0 = NEGC ? 0.f : (KBIAS ? -INFINITY : -1e30f);   // running-max start
    const float sc_l2 = KBIAS ? 1.0f : scale_log2;   // KBIAS: s already in the log2 domain
    float m_run[2] = {M0, M0}, l_run[2] = {0.f, 0.f};
    f32x4 negm[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};

    for (int t = 0; t < ntiles; ++t) {
        if (!RES && t + 1 < ntiles && !C2D_ABL(abl, 1)) gload(t + 1);
        const char* Kt = Ks + (RES ? t * SLOT : 0);
        const char* Vt = Vs + (RES ? t * SLOT : 0);

        // ---- S^T tiles: s[qg][kg] holds keys 16 kg + 4 g + r of query li
        f32x4 s[2][4], st[2][4];
#pragma unroll
        for (int qg = 0; qg < 2; ++qg)
#pragma unroll
            for (int kg = 0; kg < 4; ++kg) s[qg][kg] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kg = 0; kg < 4; ++kg) {
#pragma unroll
            for (int dc = 0; dc < C::NDC_FULL; ++dc) {
                const f16x8 kf = *reinterpret_cast<const f16x8*>(Kt + k_off<D>(kg * 16 + li, dc * 4 + g));
#pragma unroll
                for (int qg = 0; qg < 2; ++qg)
                    s[qg][kg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[qg][dc],
                                                                        (NEGC && dc == 0) ? negm[qg] : s[qg][kg],
                                                                        0, 0, 0);
            }
#pragma unroll
            for (int c = 0; c < C::NC16; ++c) {
                const f16x4 kt = *reinterpret_cast<const f16x4*>(Kt + (kg * 16 + li) * C::KS + c * 32 + g * 8);
#pragma unroll
                for (int qg = 0; qg < 2; ++qg)
                    s[qg][kg] = __builtin_amdgcn_mfma_f32_16x16x16f16(kt, q16[qg][c], s[qg][kg], 0, 0, 0);
            }
            if (C::TAIL) {
                const f16x4 kt = *reinterpret_cast<const f16x4*>(Kt + (kg * 16 + li) * C::KS + C::NDC * 64 + g * 8);
#pragma unroll
                for (int qg = 0; qg < 2; ++qg)
                    st[qg][kg] = __builtin_amdgcn_mfma_f32_16x16x16f16(kt, qt[qg], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            }
        }
        if (C::TAIL) {
#pragma unroll
            for (int qg = 0; qg < 2; ++qg)
#pragma unroll
                for (int kg = 0; kg < 4; ++kg) s[qg][kg] += st[qg][kg];
        }
        if (KBIAS) {   // additive score bias (lane holds keys 16 kg + 4 g + r of query q0 + 16 qg + li)
            const float* kbb = kbias + (size_t)b * kb_ldb + (size_t)h * kb_ldh;
#pragma unroll
            for (int qg = 0; qg < 2; ++qg) {
                const float* kbr = kbb + (size_t)min(q0 + qg * 16 + li, lq - 1) * kb_ldq;
#pragma unroll
                for (int kg = 0; kg < 4; ++kg)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int key = t * 64 + kg * 16 + g * 4 + r;
                        const float bb = key < lk ? kbr[key] : -INFINITY;
                        const float b2 = bb == -INFINITY ? bb : fmaxf(bb * kb_mul, -3.402823466e38f);
                        s[qg][kg][r] = fmaf(s[qg][kg][r], scale_log2, b2);
                    }
            }
        }
        if (MASK && (t + 1) * 64 > lk) {  // tail tile: mask keys >= lk
#pragma unroll
            for (int kg = 0; kg < 4; ++kg)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = t * 64 + kg * 16 + g * 4 + r;
                    if (key >= lk) { s[0][kg][r] = KBIAS ? -INFINITY : -1e30f; s[1][kg][r] = KBIAS ? -INFINITY : -1e30f; }
                }
        }

        // ---- online softmax (log2 domain), P packed to fp16 B fragments
        f16x8 pf[2][2];
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) {
            // lazy rescale: the running max only moves (and O, l get rescaled) when
            // some query of the wave gains more than 2^8; otherwise P <= 256 in fp16
            if (NEGC) {
                // s already holds log2-domain scores minus m_run; the first tile rebases
                // m_run (0 so far) to the tile max, later ones only move it up.  Whether any
                // row max exceeds 8 is decided on the lane maxima (same ballot); the row max
                // itself (two lane swaps) is formed only when a rescale happens
                const float lmx = lane_max16(s[qg]);
                if (t == 0 || __builtin_amdgcn_ballot_w64(lmx > 8.0f)) {
                    const float mx = quad_max(lmx);
                    const float delta = t == 0 ? mx : fmaxf(mx, 0.f);
                    const float alpha = __builtin_amdgcn_exp2f(-delta);
                    m_run[qg] += delta;
                    negm[qg] = (f32x4){-m_run[qg], -m_run[qg], -m_run[qg], -m_run[qg]};
                    if (!C::SUM_MFMA) l_run[qg] *= alpha;
#pragma unroll
                    for (int dt = 0; dt < C::NDT; ++dt) acc[dt][qg] *= alpha;
#pragma unroll
                    for (int kg = 0; kg < 4; ++kg) s[qg][kg] -= delta;
                }
            } else {
                const float mx = quad_max(lane_max16(s[qg]));
                const float m_cand = fmaxf(m_run[qg], mx * sc_l2);
                if (__builtin_amdgcn_ballot_w64(m_cand > m_run[qg] + 8.0f)) {
                    // (KBIAS: a row whose scores are all -inf so far keeps alpha = 1, its O and l are 0)
                    const float alpha = (KBIAS && m_cand == -INFINITY) ? 1.0f
                                                                        : __builtin_amdgcn_exp2f(m_run[qg] - m_cand);
                    m_run[qg] = m_cand;
                    if (!C::SUM_MFMA) l_run[qg] *= alpha;
#pragma unroll
                    for (int dt = 0; dt < C::NDT; ++dt) acc[dt][qg] *= alpha;
                }
            }
            const float m_use = (KBIAS && m_run[qg] == -INFINITY) ? 0.f : m_run[qg];
            float rs = 0.f;
#pragma unroll
            for (int kg = 0; kg < 4; ++kg)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = NEGC ? __builtin_amdgcn_exp2f(s[qg][kg][r])
                                          : __builtin_amdgcn_exp2f(fmaf(s[qg][kg][r], sc_l2, -m_use));
                    s[qg][kg][r] = pv;
                    if (!C::SUM_MFMA) rs += pv;
                }
            if (!C::SUM_MFMA) l_run[qg] += rs;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    pf[qg][kb][j] = (f16)s[qg][2 * kb][j];
                    pf[qg][kb][4 + j] = (f16)s[qg][2 * kb + 1][j];
                }
            }
        }

        // ---- O^T += V^T P^T ; V^T fragment via transposed LDS reads
#pragma unroll
        for (int dt = 0; dt < C::NDT; ++dt) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const int qq = li >> 2, pp = li & 3;
                const int row1 = kb * 32 + g * 4 + qq;
                const char* a1 = Vt + row1 * C::VS + (dt * 16 + pp * 4) * 2;
                const char* a2 = a1 + 16 * C::VS;
                s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(LDS_AS char*)a1);
                s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(LDS_AS char*)a2);
                f16x8 vf;
                f16x4 h1 = __builtin_bit_cast(f16x4, t1), h2 = __builtin_bit_cast(f16x4, t2);
#pragma unroll
                for (int j = 0; j < 4; ++j) { vf[j] = h1[j]; vf[4 + j] = h2[j]; }
#pragma unroll
                for (int qg = 0; qg < 2; ++qg)
                    acc[dt][qg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[qg][kb], acc[dt][qg], 0, 0, 0);
            }
        }

        // abl (C2D_ATTN_ABL=1): timing only, K/V tile 0 reused -- the restaging
        // costs ~17 % of the d = 40 kernel.  A two-slot LDS ring with one barrier per
        // tile (loop unrolled by two so the slot offsets fold into the ds_read
        // immediates) measured no faster at d = 40, 3 % faster at d = 80 and 10 %
        // slower on the 77-key cross-attention: the cost is the gload / swrite
        // instructions, not the second barrier.
        if (!RES && t + 1 < ntiles && !C2D_ABL(abl, 1)) {
            __syncthreads();
            swrite(0);
            __syncthreads();
        }
    }

    // ---- epilogue: lane holds O[query li][d = 16 dt + 4 g + r]
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
        float l;
        if (C::SUM_MFMA) {
            // row sum sits in O^T column D: d-tile D/16, lane group (D%16)/4, element D%4
            l = __shfl(acc[D / 16][qg][D % 4], li + 16 * ((D % 16) / 4));
        } else {
            l = l_run[qg];
            l += __shfl_xor(l, 16);
            l += __shfl_xor(l, 32);
        }
        const float inv = 1.0f / l;
        const int qi = q0 + qg * 16 + li;
        if (qi >= lq) continue;
        f16* orow = o + ((size_t)b * lq + qi) * ldo + h * D;
#pragma unroll
        for (int dt = 0; dt < C::NDT; ++dt) {
            const int d0 = dt * 16 + g * 4;
            if (d0 < D) {
                f16x4 ov;
#pragma unroll
                for (int r = 0; r < 4; ++r) ov[r] = (f16)(acc[dt][qg][r] * inv);
                *reinterpret_cast<f16x4*>(orow + d0) = ov;
            }
        }
    }
    }  // query blocks
}

// Short-sequence attention (L <= 128 keys, d = 64) with an optional causal mask:
// the CLIP ViT-L/14 text tower (77 tokens, 12 heads; transformers CLIPAttention with
// its causal mask) that produces SD1.5's encoder_hidden_states once per request.
// One workgroup per (image, head): K and V of the head staged in LDS (read as
// broadcasts: every thread walks the same key at the same time), one
// thread per query with its row in registers and an exact online softmax in fp32.
// ~0.6 MFLOP per (image, head): latency work, not worth an MFMA tile.
template <int D>
__global__ void __launch_bounds__(128) attn_small_kernel(const f16* __restrict__ q, int ldq, const f16* __restrict__ k,
                                                         int ldk, const f16* __restrict__ v, int ldv,
                                                         f16* __restrict__ o, int ldo, int heads, int l, float scale,
                                                         int causal) {
    __shared__ f16 ks[128][D], vs[128][D];
    const int bh = blockIdx.x, b = bh / heads, h = bh - b * heads;
    const int tid = threadIdx.x;
    for (int idx = tid; idx < l * D; idx += 128) {
        const int j = idx / D, c = idx - j * D;
        ks[j][c] = k[((size_t)b * l + j) * ldk + h * D + c];
        vs[j][c] = v[((size_t)b * l + j) * ldv + h * D + c];
    }
    __syncthreads();
    if (tid >= l) return;
    float qr[D], acc[D];
#pragma unroll
    for (int c = 0; c < D; ++c) {
        qr[c] = (float)q[((size_t)b * l + tid) * ldq + h * D + c] * scale;
        acc[c] = 0.f;
    }
    float m = -INFINITY, s = 0.f;
    const int jn = causal ? tid + 1 : l;
    for (int j = 0; j < jn; ++j) {
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < D; ++c) d = fmaf(qr[c], (float)ks[j][c], d);
        const float mn = fmaxf(m, d);
        const float a = __expf(m - mn), p = __expf(d - mn);
        s = s * a + p;
#pragma unroll
        for (int c = 0; c < D; ++c) acc[c] = fmaf(acc[c], a, p * (float)vs[j][c]);
        m = mn;
    }
    const float inv = 1.0f / s;
    f16* orow = o + ((size_t)b * l + tid) * ldo + h * D;
#pragma unroll
    for (int c = 0; c < D; ++c) orow[c] = (f16)(acc[c] * inv);
}

// ---------------------------------------------------------------------------
// Software-pipelined variant for d <= 64 (DP = 64: d = 40, 64).  Same fragment
// layouts as attn_fwd_kernel, but K/V tiles are double-buffered in LDS and each
// iteration issues the QK^T MFMAs of tile t+1 and the PV MFMAs of tile t, with
// the softmax of tile t+1 (VALU: max, exp2, pack) placed between the PV MFMAs so
// a wave's matrix and vector pipes overlap (the d = 40 kernel is exp-bound: PMC
// showed MFMA ~40 % and VALU ~47 % busy, executed back to back).  The online-
// softmax rescale of tile t+1 is applied after the PV of tile t retires.
template <int D, bool MASK>
__global__ void __launch_bounds__(256) attn_pp_kernel(const f16* __restrict__ q, int ldq, const f16* __restrict__ k,
                                                      int ldk, const f16* __restrict__ v, int ldv, f16* __restrict__ o,
                                                      int ldo, int heads, int lq, int lk, float scale_log2,
                                                      int kv_div, int nqb) {
    using C = AttnCfg<D>;
    static_assert(C::KSW && C::NDC_FULL == 2 && !C::TAIL, "pipelined attention: DP = 64 only");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // buffer bb: K at smem + bb * K_BYTES, V at smem + 2 * K_BYTES + bb * V_BYTES
#define KB(bb) (smem + (bb) * C::K_BYTES)
#define VB(bb) (smem + 2 * C::K_BYTES + (bb) * C::V_BYTES)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = tile / nqb, qb = tile - bh * nqb;
    const int b = bh / heads, h = bh - b * heads;
    const int bk = b / kv_div;
    const int q0 = qb * 128 + wave * 32;
    const int g = lane >> 4, li = lane & 15;

    // pads of both buffers: K chunks >= DCH zero; V pad columns zero except the ones column at D
#pragma unroll
    for (int bb = 0; bb < 2; ++bb) {
        for (int idx = tid; idx < 64 * (C::DP / 8 - C::DCH); idx += 256) {
            const int row = idx / (C::DP / 8 - C::DCH), ch = C::DCH + idx % (C::DP / 8 - C::DCH);
            *reinterpret_cast<f16x8*>(KB(bb) + k_off<D>(row, ch)) = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
        }
        for (int idx = tid; idx < 64 * (C::DV / 8 - C::DCH); idx += 256) {
            const int row = idx / (C::DV / 8 - C::DCH), ch = C::DCH + idx % (C::DV / 8 - C::DCH);
            f16x8 z = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
            if (ch == C::DCH) z[0] = (f16)1.0f;
            *reinterpret_cast<f16x8*>(VB(bb) + row * C::VS + ch * 16) = z;
        }
    }

    f16x8 qf[2][2];
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
        const int qi = q0 + qg * 16 + li;
#pragma unroll
        for (int dc = 0; dc < 2; ++dc) {
            const int d0 = dc * 32 + g * 8;
            if (qi < lq && d0 < D)
                qf[qg][dc] = *reinterpret_cast<const f16x8*>(q + ((size_t)b * lq + qi) * ldq + h * D + d0);
            else
                qf[qg][dc] = (f16x8){0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    f32x4 acc[C::NDT][2];
#pragma unroll
    for (int dt = 0; dt < C::NDT; ++dt)
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) acc[dt][qg] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float m_run[2] = {-1e30f, -1e30f};

    const f16* kbase = k + (size_t)bk * lk * ldk + h * D;
    const f16* vbase = v + (size_t)bk * lk * ldv + h * D;
    f16x8 rk[C::NLD], rv[C::NLD];
    auto gload = [&](int t) {
#pragma unroll
        for (int i = 0; i < C::NLD; ++i) {
            const int idx = tid + 256 * i;
            const int row = idx / C::DCH, ch = idx - row * C::DCH;
            const int key = min(t * 64 + row, lk - 1);   // past lk: masked scores, P = 0
            if (256 * i < 64 * C::DCH - 255 || idx < 64 * C::DCH) {
                rk[i] = *reinterpret_cast<const f16x8*>(kbase + (size_t)key * ldk + ch * 8);
                rv[i] = *reinterpret_cast<const f16x8*>(vbase + (size_t)key * ldv + ch * 8);
            }
        }
    };
    auto swrite = [&](int bb) {
#pragma unroll
        for (int i = 0; i < C::NLD; ++i) {
            const int idx = tid + 256 * i;
            if (256 * i < 64 * C::DCH - 255 || idx < 64 * C::DCH) {
                const int row = idx / C::DCH, ch = idx - row * C::DCH;
                *reinterpret_cast<f16x8*>(KB(bb) + k_off<D>(row, ch)) = rk[i];
                *reinterpret_cast<f16x8*>(VB(bb) + row * C::VS + ch * 16) = rv[i];
            }
        }
    };
    // S^T tiles of K tile in buffer bb: s[qg][kg] = keys 16 kg + 4 g + r of query li
    auto qk = [&](f32x4 (&s)[2][4], int bb) {
#pragma unroll
        for (int qg = 0; qg < 2; ++qg)
#pragma unroll
            for (int kg = 0; kg < 4; ++kg) s[qg][kg] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kg = 0; kg < 4; ++kg)
#pragma unroll
            for (int dc = 0; dc < 2; ++dc) {
                const f16x8 kf = *reinterpret_cast<const f16x8*>(KB(bb) + k_off<D>(kg * 16 + li, dc * 4 + g));
#pragma unroll
                for (int qg = 0; qg < 2; ++qg)
                    s[qg][kg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[qg][dc], s[qg][kg], 0, 0, 0);
            }
    };
    // online softmax of one tile (log2 domain, lazy 2^8 rescale): P fragments + the
    // per-query-group rescale factor to apply to O once the previous PV retired
    auto softmax = [&](f32x4 (&s)[2][4], f16x8 (&pf)[2][2], float (&alpha)[2], int t) {
        if (MASK && (t + 1) * 64 > lk) {
#pragma unroll
            for (int kg = 0; kg < 4; ++kg)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = t * 64 + kg * 16 + g * 4 + r;
                    if (key >= lk) { s[0][kg][r] = -1e30f; s[1][kg][r] = -1e30f; }
                }
        }
#pragma unroll
        for (int qg = 0; qg < 2; ++qg) {
            float mx = s[qg][0][0];
#pragma unroll
            for (int kg = 0; kg < 4; ++kg)
#pragma unroll
                for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[qg][kg][r]);
            mx = fmaxf(mx, __shfl_xor(mx, 16));
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            // branch-free lazy rescale (keeps the pipelined block one scheduling region)
            const float m_cand = fmaxf(m_run[qg], mx * scale_log2);
            const bool up = __builtin_amdgcn_ballot_w64(m_cand > m_run[qg] + 8.0f) != 0;
            const float m_new = up ? m_cand : m_run[qg];
            alpha[qg] = __builtin_amdgcn_exp2f(m_run[qg] - m_new);
            m_run[qg] = m_new;
            const float m_use = m_new;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    pf[qg][kb][j] = (f16)__builtin_amdgcn_exp2f(fmaf(s[qg][2 * kb][j], scale_log2, -m_use));
                    pf[qg][kb][4 + j] = (f16)__builtin_amdgcn_exp2f(fmaf(s[qg][2 * kb + 1][j], scale_log2, -m_use));
                }
        }
    };
    // O^T += V^T P^T for the V tile in buffer bb
    auto pv = [&](const f16x8 (&pf)[2][2], int bb) {
#pragma unroll
        for (int dt = 0; dt < C::NDT; ++dt)
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const int qq = li >> 2, pp = li & 3;
                const int row1 = kb * 32 + g * 4 + qq;
                const char* a1 = VB(bb) + row1 * C::VS + (dt * 16 + pp * 4) * 2;
                const char* a2 = a1 + 16 * C::VS;
                s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(LDS_AS char*)a1);
                s16x4 t2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(LDS_AS char*)a2);
                f16x8 vf;
                f16x4 h1 = __builtin_bit_cast(f16x4, t1), h2 = __builtin_bit_cast(f16x4, t2);
#pragma unroll
                for (int j = 0; j < 4; ++j) { vf[j] = h1[j]; vf[4 + j] = h2[j]; }
#pragma unroll
                for (int qg = 0; qg < 2; ++qg)
                    acc[dt][qg] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vf, pf[qg][kb], acc[dt][qg], 0, 0, 0);
            }
    };

    const int ntiles = (lk + 63) / 64;
    // prologue: tiles 0 and 1 staged, softmax of tile 0 done, tile 2 in registers
    gload(0);
    __syncthreads();   // pad zeroing done
    swrite(0);
    if (ntiles > 1) { gload(1); swrite(1); }
    __syncthreads();
    if (ntiles > 2) gload(2);
    f16x8 pcur[2][2], pnxt[2][2];
    {
        f32x4 s0[2][4];
        float a0[2];
        qk(s0, 0);
        softmax(s0, pcur, a0, 0);   // acc is zero: no rescale needed
    }
    for (int t = 0; t < ntiles; ++t) {
        const int cb = t & 1;
        if (t + 1 < ntiles) {
            f32x4 sn[2][4];
            float an[2];
            qk(sn, cb ^ 1);             // MFMA: scores of tile t+1
            pv(pcur, cb);               // MFMA: O += P(t) V(t)
            softmax(sn, pnxt, an, t + 1);   // VALU, overlaps the PV MFMAs in flight
            // interleave: K-fragment reads + QK^T MFMAs, then each PV MFMA (with its
            // two transposed V reads) followed by a slice of the softmax VALU work
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 8, 0);
            }
#pragma unroll
            for (int qg = 0; qg < 2; ++qg)
#pragma unroll
                for (int dt = 0; dt < C::NDT; ++dt) acc[dt][qg] *= an[qg];
#pragma unroll
            for (int qg = 0; qg < 2; ++qg)
#pragma unroll
                for (int kb = 0; kb < 2; ++kb) pcur[qg][kb] = pnxt[qg][kb];
        } else {
            pv(pcur, cb);
        }
        if (t + 2 < ntiles) {
            __syncthreads();            // every wave is done with buffer cb (K(t), V(t))
            swrite(cb);                 // tile t+2
            __syncthreads();
            if (t + 3 < ntiles) gload(t + 3);
        }
    }

    // epilogue: lane holds O[query li][d = 16 dt + 4 g + r]; row sum in the ones column D
#pragma unroll
    for (int qg = 0; qg < 2; ++qg) {
        const float l = __shfl(acc[D / 16][qg][D % 4], li + 16 * ((D % 16) / 4));
        const float inv = 1.0f / l;
        const int qi = q0 + qg * 16 + li;
        if (qi >= lq) continue;
        f16* orow = o + ((size_t)b * lq + qi) * ldo + h * D;
#pragma unroll
        for (int dt = 0; dt < C::NDT; ++dt) {
            const int d0 = dt * 16 + g * 4;
            if (d0 < D) {
                f16x4 ov;
#pragma unroll
                for (int r = 0; r < 4; ++r) ov[r] = (f16)(acc[dt][qg][r] * inv);
                *reinterpret_cast<f16x4*>(orow + d0) = ov;
            }
        }
    }
}

#undef KB
#undef VB

// C2D_TUNE_ATTN_PP=1 (variant build) selects the double-buffered, software-pipelined d=40 kernel.  Measured
// slower than the single-buffered one on MI355X (L0 self 4096x4096: 779 vs 653 us): the
// in-flight S tile takes it to 148 VGPR + 24 AGPR = 2 waves/SIMD vs 126 + 40 = 3 for
// attn_fwd_kernel<40>, and the doubled K/V ring halves the blocks LDS admits, so it is
// off by default.
// A/B constants (common.h, variant builds): C2D_TUNE_ATTN_NEGC=0 (fma-per-score softmax),
// C2D_TUNE_ATTN_RES=0 (stream K/V tiles for short key sequences too), C2D_TUNE_ATTN_W8=0
// (4-wave d = 40 blocks), C2D_TUNE_ATTN_PP=1 (the pipelined d = 40 kernel above); the timing
// ablation C2D_ATTN_ABL (K/V staging skipped) exists in the ablation build only
static int attn_abl() { return ablation_attn(); }
static bool attn_negc() { return tuning().attn_negc != 0; }
static bool attn_res() { return tuning().attn_res != 0; }
static bool attn_w8() { return tuning().attn_w8 != 0; }
static int attn_pipelined() { return tuning().attn_pp; }

// attention with an additive per-key bias: the fma-softmax kernels (resident K/V for
// lk <= 128, streaming otherwise); the bias enters in log2 units (kb_mul = log2 e)
template <int D>
static int launch_attn_bias(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                            int batch, int heads, int lq, int lk, float scale, int kv_div, const float* kbias,
                            int kb_ldb, int kb_ldh, int kb_ldq, hipStream_t s) {
    using C = AttnCfg<D>;
    const int nqb = (lq + 127) / 128;
    const int smem = C::K_BYTES + C::V_BYTES;
    const float sl2 = scale * 1.4426950408889634f, mul = 1.4426950408889634f;
    if (lk <= 128) {
        const long bhs = (long)batch * heads;
        int qpb = (int)((bhs * nqb) / 1024);
        qpb = qpb < 1 ? 1 : qpb > nqb ? nqb : qpb;
        const int ngrp = (nqb + qpb - 1) / qpb;
        dim3 g2((unsigned)(ngrp * bhs));
        hipLaunchKernelGGL((attn_fwd_kernel<D, true, false, true, true>), g2, dim3(256), 2 * smem, s, (const f16*)q,
                           ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk, sl2, kv_div, nqb,
                           0, qpb, kbias, kb_ldb, kb_ldh, mul, kb_ldq);
    } else {
        hipLaunchKernelGGL((attn_fwd_kernel<D, true, false, false, true>), dim3(nqb * batch * heads), dim3(256), smem,
                           s, (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk,
                           sl2, kv_div, nqb, 0, 1, kbias, kb_ldb, kb_ldh, mul, kb_ldq);
    }
    return check_launch();
}

template <int D>
static int launch_attn(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o, int ldo,
                       int batch, int heads, int lq, int lk, float scale, int kv_div, hipStream_t s) {
    using C = AttnCfg<D>;
    const int nqb = (lq + 127) / 128;
    const int smem = C::K_BYTES + C::V_BYTES;
    dim3 grid(nqb * batch * heads);
    if constexpr (C::KSW && C::SUM_MFMA) {
        if (attn_pipelined()) {
            const int smem2 = 2 * (C::K_BYTES + C::V_BYTES);
            if (lk % 64 == 0)
                hipLaunchKernelGGL((attn_pp_kernel<D, false>), grid, dim3(256), smem2, s, (const f16*)q, ldq,
                                   (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk,
                                   scale * 1.4426950408889634f, kv_div, nqb);
            else
                hipLaunchKernelGGL((attn_pp_kernel<D, true>), grid, dim3(256), smem2, s, (const f16*)q, ldq,
                                   (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk,
                                   scale * 1.4426950408889634f, kv_div, nqb);
            return check_launch();
        }
    }
    if (lk <= 128 && attn_res()) {
        // K/V resident, several query blocks per workgroup while >= ~1024 workgroups remain
        const long bhs = (long)batch * heads;
        int qpb = (int)((bhs * nqb) / 1024);
        qpb = qpb < 1 ? 1 : qpb > nqb ? nqb : qpb;
        const int ngrp = (nqb + qpb - 1) / qpb;
        dim3 g2((unsigned)(ngrp * bhs));
        if (lk % 64 == 0)
            hipLaunchKernelGGL((attn_fwd_kernel<D, false, false, true>), g2, dim3(256), 2 * smem, s, (const f16*)q,
                               ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk,
                               scale * 1.4426950408889634f, kv_div, nqb, 0, qpb);
        else
            hipLaunchKernelGGL((attn_fwd_kernel<D, true, false, true>), g2, dim3(256), 2 * smem, s, (const f16*)q,
                               ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk,
                               scale * 1.4426950408889634f, kv_div, nqb, 0, qpb);
        return check_launch();
    }
#define C2D_ATTN_LAUNCH(MASK, NEGC)                                                                             \
    hipLaunchKernelGGL((attn_fwd_kernel<D, MASK, NEGC>), grid, dim3(256), smem, s, (const f16*)q, ldq, (const f16*)k, \
                       ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, lq, lk, scale * 1.4426950408889634f, kv_div, nqb, \
                       attn_abl())
    if constexpr (D == 40) {
        // 8-wave blocks (256 queries): one K / V staging chunk per thread instead of two
        // (L0: 586-628 -> 560-594 us, same box); d = 80 measured 72 -> 76 us with them
        const int nqb8 = (lq + 255) / 256;
        if (lk % 64 == 0 && lk >= 256 && attn_negc() && attn_w8() && nqb8 * batch * heads >= C2D_TUNE_ATTN_W8_MIN) {
            hipLaunchKernelGGL((attn_fwd_kernel<D, false, true, false, false, 8>), dim3(nqb8 * batch * heads),
                               dim3(512), smem, s, (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o,
                               ldo, heads, lq, lk, scale * 1.4426950408889634f, kv_div, nqb8, attn_abl());
            return check_launch();
        }
    }
    // NEGC pays its Q pre-scale and peeled first tile back only over several key tiles
    // (measured: 4096 keys d = 40 681 -> 646 us, d = 80 75.7 -> 72.6; 77 keys 35.8 -> 38.4)
    const bool mask = lk % 64 != 0, negc = attn_negc() && lk >= 256;
    if (!mask && negc) C2D_ATTN_LAUNCH(false, true);
    else if (!mask) C2D_ATTN_LAUNCH(false, false);
    else if (negc) C2D_ATTN_LAUNCH(true, true);
    else C2D_ATTN_LAUNCH(true, false);
#undef C2D_ATTN_LAUNCH
    return check_launch();
}

// ------------------------------------------------------------ window attention
// one workgroup of 64 threads per (window, head); thread = query.  d <= 32.
__global__ void __launch_bounds__(64) window_attn_kernel(const f16* __restrict__ qkv, int ld, const int* __restrict__ row_map,
                                                         int heads, int d, const float* __restrict__ bias,
                                                         const float* __restrict__ mask, int n_mask,
                                                         f16* __restrict__ out, int ldo, float scale) {
    __shared__ float Ks[64][33];
    __shared__ float Vs[64][33];
    const int w = blockIdx.x / heads, h = blockIdx.x - (blockIdx.x / heads) * heads;
    const int t = threadIdx.x;
    const int C = heads * d;
    const int row = row_map[w * 64 + t];
    const f16* base = qkv + (size_t)row * ld;
    float qv[32];
    for (int i = 0; i < d; ++i) {
        qv[i] = (float)base[h * d + i] * scale;
        Ks[t][i] = (float)base[C + h * d + i];
        Vs[t][i] = (float)base[2 * C + h * d + i];
    }
    __syncthreads();
    const float* brow = bias + ((size_t)h * 64 + t) * 64;
    const float* mrow = mask ? mask + ((size_t)(w % n_mask) * 64 + t) * 64 : nullptr;
    float sc[64];
    float mx = -1e30f;
    for (int j = 0; j < 64; ++j) {
        float a = 0.f;
        for (int i = 0; i < d; ++i) a = fmaf(qv[i], Ks[j][i], a);
        a += brow[j];
        if (mrow) a += mrow[j];
        sc[j] = a;
        mx = fmaxf(mx, a);
    }
    float l = 0.f;
    for (int j = 0; j < 64; ++j) { sc[j] = __expf(sc[j] - mx); l += sc[j]; }
    const float inv = 1.0f / l;
    f16* orow = out + (size_t)row * ldo + h * d;
    for (int i = 0; i < d; ++i) {
        float a = 0.f;
        for (int j = 0; j < 64; ++j) a = fmaf(sc[j], Vs[j][i], a);
        orow[i] = (f16)(a * inv);
    }
}

}  // namespace c2d

using namespace c2d;

extern "C" int c2d_attention_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                                 int ldo, int batch, int heads, int lq, int lk, int d, float scale, int kv_div,
                                 void* stream) {
    if (!q || !k || !v || !o || kv_div <= 0) return C2D_E_ARG;
    if (batch <= 0 || heads <= 0 || lq <= 0 || lk <= 0) return C2D_E_SHAPE;
    if ((ldq & 7) || (ldk & 7) || (ldv & 7) || (ldo & 3)) return C2D_E_ALIGN;
    if (!aligned16(q) || !aligned16(k) || !aligned16(v) || ((uintptr_t)o & 7)) return C2D_E_ALIGN;
    if (heads * d > ldq || heads * d > ldk || heads * d > ldv || heads * d > ldo) return C2D_E_SHAPE;
    hipStream_t s = (hipStream_t)stream;
    switch (d) {
        case 40: return launch_attn<40>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, scale, kv_div, s);
        case 64: return launch_attn<64>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, scale, kv_div, s);
        case 80: return launch_attn<80>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, scale, kv_div, s);
        case 160: return launch_attn<160>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, scale, kv_div, s);
        default: return C2D_E_SHAPE;
    }
}

extern "C" int c2d_attention_fwd_mask(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                      void* o, int ldo, int batch, int heads, int lq, int lk, int d, float scale,
                                      int kv_div, const float* bias, int bias_ld_batch, int bias_ld_head,
                                      int bias_ld_query, void* stream) {
    if (!bias) return c2d_attention_fwd(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, d, scale, kv_div,
                                        stream);
    if (!q || !k || !v || !o || kv_div <= 0) return C2D_E_ARG;
    if (batch <= 0 || heads <= 0 || lq <= 0 || lk <= 0 || scale == 0.f) return C2D_E_SHAPE;
    if (bias_ld_batch < 0 || bias_ld_head < 0 || bias_ld_query < 0) return C2D_E_SHAPE;
    if ((ldq & 7) || (ldk & 7) || (ldv & 7) || (ldo & 3)) return C2D_E_ALIGN;
    if (!aligned16(q) || !aligned16(k) || !aligned16(v) || ((uintptr_t)o & 7)) return C2D_E_ALIGN;
    if (heads * d > ldq || heads * d > ldk || heads * d > ldv || heads * d > ldo) return C2D_E_SHAPE;
    hipStream_t s = (hipStream_t)stream;
#define C2D_ATTN_B(DD) launch_attn_bias<DD>(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, scale, kv_div, \
                                            bias, bias_ld_batch, bias_ld_head, bias_ld_query, s)
    switch (d) {
        case 40: return C2D_ATTN_B(40);
        case 64: return C2D_ATTN_B(64);
        case 80: return C2D_ATTN_B(80);
        case 160: return C2D_ATTN_B(160);
        default: return C2D_E_SHAPE;
    }
#undef C2D_ATTN_B
}

extern "C" int c2d_attention_fwd_bias(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                                      void* o, int ldo, int batch, int heads, int lq, int lk, int d, float scale,
                                      int kv_div, const float* key_bias, int bias_ld_batch, int bias_ld_head,
                                      void* stream) {
    return c2d_attention_fwd_mask(q, ldq, k, ldk, v, ldv, o, ldo, batch, heads, lq, lk, d, scale, kv_div, key_bias,
                                  bias_ld_batch, bias_ld_head, 0, stream);
}

extern "C" int c2d_window_attention(const void* qkv, int ld_qkv, const int* row_map, int n_windows, int heads, int d,
                                    const float* bias, const float* mask, int n_mask, void* out, int ldo,
                                    void* stream) {
    if (!qkv || !row_map || !bias || !out) return C2D_E_ARG;
    if (d <= 0 || d > 32 || heads <= 0 || n_windows <= 0) return C2D_E_SHAPE;
    if (mask && n_mask <= 0) return C2D_E_ARG;
    if (ld_qkv < 3 * heads * d || ldo < heads * d) return C2D_E_SHAPE;
    hipLaunchKernelGGL(window_attn_kernel, dim3(n_windows * heads), dim3(64), 0, (hipStream_t)stream,
                       (const f16*)qkv, ld_qkv, row_map, heads, d, bias, mask, n_mask, (f16*)out, ldo,
                       1.0f / sqrtf((float)d));
    return check_launch();
}

extern "C" int c2d_attention_small(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                                   int ldo, int batch, int heads, int l, int d, float scale, int causal,
                                   void* stream) {
    if (!q || !k || !v || !o) return C2D_E_ARG;
    if (d != 64 || l <= 0 || l > 128 || batch < 0 || heads <= 0) return C2D_E_SHAPE;
    if (batch == 0) return 0;
    hipLaunchKernelGGL(attn_small_kernel<64>, dim3(batch * heads), dim3(128), 0, (hipStream_t)stream,
                       (const f16*)q, ldq, (const f16*)k, ldk, (const f16*)v, ldv, (f16*)o, ldo, heads, l, scale,
                       causal);
    return check_launch();
}
