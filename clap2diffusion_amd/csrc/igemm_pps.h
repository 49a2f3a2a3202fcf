// Persistent ping-pong 1x1 GEMM with a carried epilogue (tile 50; included by igemm.hip
// after igemm_pp16.h; uses IgemmParams, M32Loader, lds_sw, wait_vm_c, make_rsrc, kOOB).
//
// Why: on the K = 320 / 640 / 1280 projections of the transformer blocks (GEGLU, QKV,
// to_q, proj_in) a 256-row tile has 5-20 K steps, and its epilogue -- bias, GEGLU's
// h * gelu(g), the fp16 stores -- ran after the K loop on every CU at once: the timing
// ablation of the one-shot ping-pong / 32x32 kernels (profiles/r03_pp16_ablation.txt)
// put it at 46 % of the L0 GEGLU (190 -> 103 us without it) and 43 % of the L0 QKV
// (70 -> 40 us), with HBM idle during the K loops and saturated by the stores of all
// 256 CUs at each round boundary.
//
// What: one workgroup per CU walks tiles t = first + i * grid.  The K loop is the
// ping-pong of igemm_pp16.h (8 waves = 2 row groups x 4 column waves, 16x16x32 MFMAs,
// LDS-DMA ring of two K-64 slots, the row groups one barrier apart) on a 192 x 256 tile
// (wave tile 96 x 64); the DMA of the next tile's first K step is dealt in the last K
// step of the current one, so the ring never drains between tiles.  At a tile's end each
// wave folds its accumulators (+ bias) into fp16 registers -- the "stash": GEGLU keeps h
// and g, a plain output its values -- and the NEXT tile's K loop, fully unrolled (NK K
// steps x 4 phases, so every stash index is a compile-time constant), spends a fixed
// share of that stash per phase inside its MFMA sections: GEGLU's h * gelu(g) on the
// VALU beside the matrix pipe, one 8-byte buffer store per 4 outputs (out-of-range rows
// pushed past num_records: no branch splits a section).  The last tile's stash is
// flushed after the loop.  Plain outputs without a residual / time embedding only.
#pragma once

#ifndef C2D_PPS_AUX
#define C2D_PPS_AUX 0   // cache policy of the carried-epilogue stores (A/B builds: 2 = nt, 16 = sc1)
#endif

namespace c2d {

template <int NK, bool GG, int PH>
__global__ void __launch_bounds__(512) igemm_pps_kernel(IgemmParams p) {
    constexpr int TN = 4, TMW = 6, BK = 64, NW = 8;
    constexpr int BM = 2 * TMW * 16, BN = 4 * TN * 16;   // 192 x 256 (a 256-row tile: 256 VGPRs + 66-129 spilled)
    constexpr int RB = 2 * BK, STAGE = (BM + BN) * RB;
    typedef M32Loader<BM, BN, BK, NW, 1> Loader;
    constexpr int P = Loader::PMAX, SA = Loader::SA, SB = Loader::SB;
    static_assert(Loader::PMIN == P, "every wave deals the same pieces");
    // PH phases per K step: 4 = (k32 half, row half) with 12-MFMA sections, 2 = k32 half with
    // 24-MFMA sections (half the barriers, all six A row tiles' fragments live; every DMA piece
    // of the next K step dealt in phase 0).  L0 GEGLU (K = 320) same box, three alternations:
    // 172.3-173.7 us with 4 phases, 165.1-166.7 with 2; K = 640 / 1280 keep 4 (2 spills 34 VGPRs)
    constexpr int RT = PH == 4 ? TMW / 2 : TMW;
    static_assert(PH == 2 || PH == 4, "pps phases per K step");
    constexpr int PPH = (P + PH - 2) / (PH - 1);   // pieces per phase, phases 0..PH-2
    constexpr int NSEC = PH * NK;        // sections (phases) per tile
    constexpr int NU = GG ? 2 * TMW : TN * TMW;   // stash units: 4 outputs (one 8-B store) per lane
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int ntiles = p.gx * p.gy, G = gridDim.x;
    int tile = xcd_remap(blockIdx.x, G);
    const int l15 = lane & 15, lg = lane >> 4;
    const int out_cols = GG ? (p.cout >> 1) : p.cout;
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out, (unsigned)((size_t)p.M * p.out_ld * 2));

    // per-tile row / column addressing of the LDS-DMA loader (1x1: the A row of output
    // pixel m is input pixel m); everything else in the loader is tile-independent
    Loader ld;
    auto tile_origin = [&](int t, int& m0, int& n0) {
        const int mt = t / p.gx;
        m0 = mt * BM;
        n0 = (t - mt * p.gx) * BN;
    };
    auto retarget = [&](int m0, int n0) {
#pragma unroll
        for (int i = 0; i < SA; ++i) {
            const int m = m0 + ld.row_of(wave, i);
            ld.a_pix[i] = m < p.M ? m : 0;
            ld.a_mask[i] = m < p.M ? 1u : 0u;
        }
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            const int row = ld.row_of(wave, i);
            const int j = n0 + row;
            ld.b_off[i] = (row < BN && j < p.cout) ? (unsigned)(2 * (j * p.kpad + ld.chunk_of(row))) : kOOB;
        }
        ld.cbase = 0;
        ld.tap = 0;
    };
    const int fo0 = lds_sw<BK>(l15, lg), fo1 = lds_sw<BK>(l15, 4 + lg);
    const int a_base = wr * TMW * 16 * RB, b_base = BM * RB + wc * TN * 16 * RB;

    // the stash of the previous tile: fp16 (bias added), in the accumulator layout
    f16x4 sh[GG ? 2 : TN][TMW], sg[GG ? 2 : 1][TMW];
#pragma unroll
    for (int b = 0; b < TMW; ++b) {
#pragma unroll
        for (int a = 0; a < (GG ? 2 : TN); ++a) sh[a][b] = (f16x4){0, 0, 0, 0};
#pragma unroll
        for (int a = 0; a < (GG ? 2 : 1); ++a) sg[a][b] = (f16x4){0, 0, 0, 0};
    }
    int prev_m = -1, prev_j = 0;   // this lane's first output row / column of the stashed tile
    auto unit = [&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        if (C2D_ABL(p.abl, 4)) return;   // timing ablation: no carried epilogue at all
        constexpr int ua = u / TMW, ub = u - (u / TMW) * TMW;
        const int m = prev_m + ub * 16;
        const int j = prev_j + ua * 16;
        const bool ok = prev_m >= 0 && m < p.M && j < out_cols;
        const unsigned off = ok ? (unsigned)(2 * (m * p.out_ld + j)) : kOOB;
        f16x4 o;
        if constexpr (GG) {
            // packed-pair math (geglu2), three alternations on one box: L0 GEGLU unchanged (161-164
            // us), L1 144-146 -> 141-142 us (profiles/r03_geglu_pk_ab.txt)
            const f32x4 hf = __builtin_convertvector(sh[ua][ub], f32x4);
            const f32x4 gf = __builtin_convertvector(sg[ua][ub], f32x4);
            const f32x2 lo = geglu2(hf.xy, gf.xy), hi = geglu2(hf.zw, gf.zw);
            o = __builtin_convertvector(((f32x4){lo.x, lo.y, hi.x, hi.y}), f16x4);
        } else {
            o = sh[ua][ub];
        }
        if (C2D_ABL(p.abl, 8)) {   // timing ablation: epilogue math kept, no store
            asm volatile("" :: "v"(o), "v"(off));
            return;
        }
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ro, (int)off, 0, C2D_PPS_AUX);
    };

    f32x4 acc[TN][TMW];
    f32x4 bv[TN];
#define C2D_BAR() do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
    int m0, n0;
    tile_origin(tile, m0, n0);
    ld.init(p, m0, n0, wave, lane, 0);
    if (tile < ntiles) ld.issue(p, 0, smem, wave);
    wait_vm_c<0>();
    C2D_BAR();
    if (wr) C2D_BAR();   // group 1 runs one barrier behind group 0

    f16x8 fa[RT], fb[TN];
    int base = 0;        // ring slot parity of this tile's K step 0
    for (; tile < ntiles; tile += G) {
        const int next = tile + G;
        const bool has_next = next < ntiles;
        static_for<0, NK>([&](auto ktc) __attribute__((always_inline)) {
            constexpr int kt = decltype(ktc)::value;
            if (kt == NK - 1) {   // the bias is live only across the last K step
#pragma unroll
                for (int a = 0; a < TN; ++a) bv[a] = bias4(p, n0 + wc * TN * 16 + a * 16 + 4 * lg);
            }
            const char* S = smem + ((base + kt) & 1) * STAGE;
            char* Wn = smem + ((base + kt + 1) & 1) * STAGE;
            const bool nxt = kt + 1 < NK || has_next;
            if (kt == NK - 1 && has_next) {   // the next K step is the next tile's step 0
                int nm0, nn0;
                tile_origin(next, nm0, nn0);
                retarget(nm0, nn0);
            }
            typename Loader::Stage st = ld.prep(p);
            static_for<0, PH>([&](auto qc) __attribute__((always_inline)) {
                constexpr int q = decltype(qc)::value;
                constexpr int ks = PH == 4 ? q >> 1 : q, rh = PH == 4 ? q & 1 : 0, sec = kt * PH + q;
                const int fo = ks ? fo1 : fo0;
                // ---- load section
                if (rh == 0) {
#pragma unroll
                    for (int t = 0; t < TN; ++t) fb[t] = *reinterpret_cast<const f16x8*>(S + b_base + t * 16 * RB + fo);
                }
#pragma unroll
                for (int t = 0; t < RT; ++t)
                    fa[t] = *reinterpret_cast<const f16x8*>(S + a_base + (rh * RT + t) * 16 * RB + fo);
                if (q < PH - 1 && nxt) {
#pragma unroll
                    for (int i = 0; i < PPH; ++i)
                        if (q * PPH + i < P) ld.piece(st, Wn, wave, q * PPH + i);
                }
                if (q == PH - 1 && nxt) wait_vm_c<0>();   // own pieces of the next K step landed
                __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
                C2D_BAR();
                // ---- MFMA section (+ this section's share of the previous tile's stash)
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int b = 0; b < RT; ++b)
#pragma unroll
                    for (int a = 0; a < TN; ++a)
                        acc[a][rh * RT + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                            fb[a], fa[b], (kt == 0 && ks == 0) ? (f32x4){0.f, 0.f, 0.f, 0.f} : acc[a][rh * RT + b],
                            0, 0, 0);
                static_for<(sec * NU) / NSEC, ((sec + 1) * NU) / NSEC>(unit);
                __builtin_amdgcn_s_setprio(0);
                C2D_BAR();
            });
            if (kt + 1 < NK) ld.advance();
        });
        // fold this tile into the stash (the next tile's sections store it)
        prev_m = m0 + wr * TMW * 16 + l15;
        prev_j = (GG ? ((n0 + wc * TN * 16) >> 1) : (n0 + wc * TN * 16)) + 4 * lg;
#pragma unroll
        for (int b = 0; b < TMW; ++b) {
            if constexpr (GG) {
#pragma unroll
                for (int pr = 0; pr < 2; ++pr) {
                    const f32x4 h = acc[2 * pr][b] + bv[2 * pr], g = acc[2 * pr + 1][b] + bv[2 * pr + 1];
#pragma unroll
                    for (int r = 0; r < 4; ++r) { sh[pr][b][r] = (f16)h[r]; sg[pr][b][r] = (f16)g[r]; }
                }
            } else {
#pragma unroll
                for (int a = 0; a < TN; ++a) {
                    const f32x4 v = acc[a][b] + bv[a];
#pragma unroll
                    for (int r = 0; r < 4; ++r) sh[a][b][r] = (f16)v[r];
                }
            }
        }
        if (has_next) {
            ld.advance();
            tile_origin(next, m0, n0);
        }
        base = (base + NK) & 1;
    }
    static_for<0, NU>(unit);   // flush the last tile's stash
    if (!wr) C2D_BAR();        // balance the stagger
#undef C2D_BAR
}

template <int NK, bool GG>
static void launch_pps(IgemmParams& p, hipStream_t s) {
    constexpr int smem = 2 * (192 + 256) * 128;
    constexpr int PH = NK == 5 ? 2 : 4;
    static_assert(smem <= 160 * 1024, "LDS ring too large");
    ensure_lds<igemm_pps_kernel<NK, GG, PH>>(smem);
    p.gx = (p.cout + 255) / 256;
    p.gy = (p.M + 191) / 192;
    const int ntiles = p.gx * p.gy;
    const int grid = ntiles < 256 ? ntiles : 256;
    hipLaunchKernelGGL((igemm_pps_kernel<NK, GG, PH>), dim3(grid), dim3(512), smem, s, p);
}

// K steps of 64 the unrolled kernel is instantiated for (K = 320 / 640 / 1280: every
// transformer-block projection of the SD1.5 UNet)
__host__ __device__ constexpr bool pps_nk_ok(int nk) { return nk == 5 || nk == 10 || nk == 20; }

static void run_pps(IgemmParams& p, hipStream_t s) {
    const bool gg = p.act == C2D_ACT_GEGLU;
    switch (p.kpad / 64) {
        case 5: return gg ? launch_pps<5, true>(p, s) : launch_pps<5, false>(p, s);
        case 10: return gg ? launch_pps<10, true>(p, s) : launch_pps<10, false>(p, s);
        default: return gg ? launch_pps<20, true>(p, s) : launch_pps<20, false>(p, s);
    }
}

}  // namespace c2d
