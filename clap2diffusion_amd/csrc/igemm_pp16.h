// Ping-pong implicit GEMM on v_mfma_f32_16x16x32_f16 (included by igemm.hip after
// igemm_m32.h; uses IgemmParams, M32Loader, lds_sw, wait_vm*, epi_pass, splitk_reduce).
//
// Structure (cdna_hip_programming.md §5, "the 256² 8-phase template", adapted to the
// implicit-GEMM conv and a 256 x 320 tile):
//   * 512 threads = 8 waves in 2 (rows) x 4 (columns); wave (wr, wc) owns output rows
//     wr*128 .. +128 and packed weight rows wc*16*TN .. +16*TN (TN = 5: 80 columns).
//   * K steps of 64 staged by LDS-DMA (M32Loader, the same lane-linear XOR-swizzled
//     [rows][64] image as the 32x32 kernels) into a 2-slot ring (144 KiB at 256 x 320).
//   * Each K step is 4 phases q = (ks, rh): k32 half ks, row half rh (4 of the wave's 8
//     16-row tiles); a phase = a LOAD section (its A fragments, the B fragments when
//     rh = 0 -- reused by the rh = 1 phase -- and up to 3 DMA pieces of the next K step)
//     and an MFMA section (4 x TN MFMAs), each closed by a workgroup barrier.
//   * The two row groups (waves 0-3, 4-7: one of each per SIMD) run one barrier apart,
//     so on every SIMD one wave issues MFMAs while the other issues its LDS reads and
//     DMA pieces: the matrix pipe never waits on the fragment-read latency or on the
//     60-185 cycles a DMA piece holds its wave's issue.
// Synchronisation (group 1 lags group 0 by one barrier):
//   RAW  the next K step's pieces are dealt in phases 0-2; every wave waits for its own
//        pieces (vmcnt(0)) at the end of its phase-3 load section, before that section's
//        barrier, which precedes every wave's first read of that K step.
//   WAR  DMA into slot (kt+1) & 1 starts in phase (kt, 0); the last reads of that slot
//        (K step kt-1, group 1's phase-3 load section) completed (lgkmcnt(0)) before the
//        barrier that ends that section, which group 0 passes before its phase (kt, 0).
// Why 16x16x32: same LDS bytes per MAC as 32x32x16 at equal wave tile, half the cycles per
// MFMA (finer interleave), and the chip holds a higher clock on it (MI355X_MICROARCH.md,
// DVFS item 7: ~1.12-1.15x the FLOP/s on random data).
#pragma once

#ifndef C2D_PP16_PH
#define C2D_PP16_PH 0   // 0: per shape family (launch_pp16); 2 / 4 force (A/B builds)
#endif
#ifndef C2D_PP16_LGKM_ALL
#define C2D_PP16_LGKM_ALL 1   // 0: lgkmcnt(0) only in phase 3 (measured neutral: bench 7.845 / 7.840 vs 7.850 / 7.837)
#endif

namespace c2d {

// Accumulators stay in the VGPR form the compiler picks.  AGPR accumulators overlap LDS
// reads with MFMAs better in isolation (scripts/microbench/mfma_lds.hip), but the 160
// accumulator registers of this tile do not fit the AGPR half the allocator grants at two
// waves per SIMD: with the AGPR-form hint it split them and copied in the loop (40 % slower),
// and inline-asm "+a" MFMAs computed wrong results (hazards invisible to the compiler).
template <int TN, int KS, int PH>
__global__ void __launch_bounds__(512) igemm_pp16_kernel(IgemmParams p) {
    constexpr int BK = 64, NW = 8, TMW = 8;
    constexpr int BM = 2 * TMW * 16, BN = 4 * TN * 16;
    constexpr int RB = 2 * BK, STAGE = (BM + BN) * RB;
    typedef M32Loader<BM, BN, BK, NW, KS> Loader;
    constexpr int P = Loader::PMAX;
    static_assert(Loader::PMIN == P, "every wave deals the same pieces");
    // PH phases per K step: 4 = (k32 half, row half), 20-MFMA sections; 2 = k32 half, 40-MFMA
    // sections (half the barriers; all eight A row tiles' fragments live; every DMA piece of
    // the next K step dealt in phase 0, so phase 1 is its landing time).  Same box, two
    // alternations over the c3 shapes (profiles/r03_pp16_phases_ab.txt): 1x1 GEMMs with
    // K >= 640 and the 256x256 tile 3-4 % faster with 2, the 256x320 3x3 convs within +-0.7 %
    constexpr int RT = PH == 4 ? 4 : 8;
    static_assert(PH == 2 || PH == 4, "pp16 phases per K step");
    constexpr int PPH = (P + PH - 2) / (PH - 1);   // pieces per phase, phases 0..PH-2
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int bid = xcd_remap(blockIdx.x, p.gx * p.gy * p.ksplit);
    const int tile = bid / p.ksplit, slice = bid - tile * p.ksplit;
    const int mt = tile / p.gx, nt = tile - mt * p.gx;
    const int m0 = mt * BM, n0 = nt * BN;
    const int nk_all = p.kpad / BK;
    const int kb = slice * p.nkt, ke = min(nk_all, kb + p.nkt);

    Loader ld;
    ld.init(p, m0, n0, wave, lane, kb);
    // fragment offsets: 16x16x32 operand = 16 rows (lane & 15) x 8 k (chunk lane >> 4) per k32
    const int fo0 = lds_sw<BK>(lane & 15, lane >> 4), fo1 = lds_sw<BK>(lane & 15, 4 + (lane >> 4));
    const int a_base = wr * TMW * 16 * RB, b_base = BM * RB + wc * TN * 16 * RB;

    f32x4 acc[TN][TMW];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TMW; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

#define C2D_BAR() do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
    if (kb < ke) ld.issue(p, kb, smem + (kb & 1) * STAGE, wave);
    wait_vm_c<0>();
    C2D_BAR();
    if (wr) C2D_BAR();   // group 1 runs one barrier behind group 0

    f16x8 fa[RT], fb[TN];
    for (int kt = kb; kt < ke; ++kt) {
        const char* S = smem + (kt & 1) * STAGE;
        char* Wn = smem + ((kt + 1) & 1) * STAGE;
        const bool nxt = kt + 1 < ke;
        typename Loader::Stage st = ld.prep(p);
#pragma unroll
        for (int q = 0; q < PH; ++q) {
            const int ks = PH == 4 ? q >> 1 : q, rh = PH == 4 ? q & 1 : 0;
            const int fo = ks ? fo1 : fo0;
            // ---- load section
            if (rh == 0) {
#pragma unroll
                for (int t = 0; t < TN; ++t) fb[t] = *reinterpret_cast<const f16x8*>(S + b_base + t * 16 * RB + fo);
            }
#pragma unroll
            for (int t = 0; t < RT; ++t)
                fa[t] = *reinterpret_cast<const f16x8*>(S + a_base + (rh * 4 + t) * 16 * RB + fo);
            if (q < PH - 1 && nxt && !C2D_ABL(p.abl, 1)) {
#pragma unroll
                for (int i = 0; i < PPH; ++i)
                    if (q * PPH + i < P) ld.piece(st, Wn, wave, q * PPH + i);
            }
            if (q == PH - 1 && nxt) wait_vm_c<0>();   // own pieces of K step kt+1 landed
            // lgkmcnt(0) before the barrier only where the WAR argument needs it (the last
            // reads of this ring slot, phase 3); in phases 0-2 the fragment reads' latency
            // runs under the barrier wait and the compiler's own wait before the first MFMA
            // that uses them (cdna_hip_programming.md 8-phase template: wait after the barrier)
            if (q == PH - 1 || C2D_PP16_LGKM_ALL)
                __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
            C2D_BAR();
            // ---- MFMA section
            if (C2D_ABL(p.abl, 2)) {   // timing ablation: fragments kept live, no MFMA
#pragma unroll
                for (int t = 0; t < RT; ++t) asm volatile("" :: "v"(fa[t]));
#pragma unroll
                for (int t = 0; t < TN; ++t) asm volatile("" :: "v"(fb[t]));
            } else {
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int b = 0; b < RT; ++b)
#pragma unroll
                    for (int a = 0; a < TN; ++a)
                        acc[a][rh * 4 + b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[a], fa[b], acc[a][rh * 4 + b], 0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
            }
            C2D_BAR();
        }
        if (nxt) ld.advance();
    }
    if (!wr) C2D_BAR();   // balance the stagger
#undef C2D_BAR

    const int mw0 = m0 + wr * TMW * 16, nw0 = n0 + wc * TN * 16;
    if (C2D_ABL(p.abl, 4)) {   // timing ablation: no epilogue (accumulators kept live)
#pragma unroll
        for (int a = 0; a < TN; ++a)
#pragma unroll
            for (int b = 0; b < TMW; ++b) asm volatile("" :: "v"(acc[a][b]));
        return;
    }
    if (p.ksplit > 1) {
#pragma unroll
        for (int b = 0; b < TMW; ++b) {
            const int m = mw0 + b * 16 + (lane & 15);
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                const int j = nw0 + a * 16 + 4 * (lane >> 4);
                if (m < p.M && j < p.cout) store_partial(p, slice, m, j, acc[a][b]);
            }
        }
        return;
    }
    // LDS-staged epilogue (epilogue.h).  Outputs with a residual or a time embedding: four
    // passes; in each every wave writes 32 of its rows (bias added) into one workgroup image
    // of 2 x 32 rows x the tile's 16 TN x 4 columns and all 512 threads finish it, each
    // chunk's residual / temb loads issued with its image read (one wait per chunk; the
    // round-1 per-chunk branches paid up to three serialised round trips).  Plain outputs:
    // the round-1 per-wave image loop (faster there, see epi_rows_plain).
    __syncthreads();
    if (!p.resid && !p.temb) {
        constexpr int PITCHF = TN * 16 + 4;
        float* img = reinterpret_cast<float*>(smem) + wave * 32 * PITCHF;
#pragma unroll
        for (int b0 = 0; b0 < TMW; b0 += 2) {
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                for (int a = 0; a < TN; ++a)
                    *reinterpret_cast<f32x4*>(img + (bb * 16 + (lane & 15)) * PITCHF + a * 16 + 4 * (lane >> 4)) =
                        acc[a][b0 + bb];
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
            epi_rows_plain<32, TN * 16>(p, img, PITCHF, mw0 + b0 * 16, nw0, lane);
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
            __builtin_amdgcn_wave_barrier();
        }
    } else if (TN == 5 && p.gn_mom) {   // + the output's GroupNorm moments (tile 40; c2d_conv_desc::gn_mom)
        constexpr int BN = 4 * TN * 16, PITCHB = BN + 4;
        float* img = reinterpret_cast<float*>(smem);
        const int wr0 = wr * 32, wc0 = wc * TN * 16;
        epi_gn_moments<TMW / 2, 64, BN, BM, TMW * 16>(p, img, PITCHB, m0, n0, tid, [&](auto pass) __attribute__((always_inline)) {
            constexpr int b0 = 2 * decltype(pass)::value;
            f32x4 bv[TN];
#pragma unroll
            for (int a = 0; a < TN; ++a) bv[a] = bias4(p, nw0 + a * 16 + 4 * (lane >> 4));
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                for (int a = 0; a < TN; ++a)
                    *reinterpret_cast<f32x4*>(img + (wr0 + bb * 16 + (lane & 15)) * PITCHB + wc0 + a * 16 +
                                              4 * (lane >> 4)) = acc[a][b0 + bb] + bv[a];
        });
    } else {
        constexpr int BN = 4 * TN * 16, PITCHB = BN + 4;
        float* img = reinterpret_cast<float*>(smem);
        const int wr0 = wr * 32, wc0 = wc * TN * 16;
        static_for<0, TMW / 2>([&](auto pass) __attribute__((always_inline)) {
            constexpr int b0 = 2 * decltype(pass)::value;
            epi_pass<64, BN, true, 512, TMW * 16>(p, img, PITCHB, m0 + b0 * 16, n0, tid, [&]() __attribute__((always_inline)) {
                f32x4 bv[TN];
#pragma unroll
                for (int a = 0; a < TN; ++a) bv[a] = bias4(p, nw0 + a * 16 + 4 * (lane >> 4));
#pragma unroll
                for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                    for (int a = 0; a < TN; ++a)
                        *reinterpret_cast<f32x4*>(img + (wr0 + bb * 16 + (lane & 15)) * PITCHB + wc0 + a * 16 +
                                                  4 * (lane >> 4)) = acc[a][b0 + bb] + bv[a];
            });
        });
    }
}

template <int TN, int KS>
static void launch_pp16(const IgemmParams& p, hipStream_t s) {
    constexpr int PH = C2D_PP16_PH ? C2D_PP16_PH : ((KS == 1 || TN == 4) ? 2 : 4);
    constexpr int ring = 2 * (256 + 4 * TN * 16) * 128;
    constexpr int epi_wg = 64 * (4 * TN * 16 + 4) * 4, epi_wv = 8 * 32 * (TN * 16 + 4) * 4;   // epilogue images
    constexpr int epi = epi_wg > epi_wv ? epi_wg : epi_wv;
    constexpr int smem = ring > epi ? ring : epi;
    static_assert(smem <= 160 * 1024, "LDS ring / epilogue image too large");
    auto k = igemm_pp16_kernel<TN, KS, PH>;
    ensure_lds<igemm_pp16_kernel<TN, KS, PH>>(smem);
    hipLaunchKernelGGL(k, dim3(p.gx * p.gy * p.ksplit), dim3(512), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

template <int TN>
static void run_pp16(IgemmParams& p, int ksize, int cout, hipStream_t s) {
    constexpr int BM = 256, BN = 4 * TN * 16;
    p.gx = (cout + BN - 1) / BN;
    p.gy = (p.M + BM - 1) / BM;
    if (ksize == 1) launch_pp16<TN, 1>(p, s);
    else launch_pp16<TN, 3>(p, s);
}

}  // namespace c2d
