// Software-pipelined implicit GEMM on v_mfma_f32_16x16x32_f16, one barrier per K step
// (tiles 60 = 256 x 320, 61 = 256 x 256; included by igemm.hip after igemm_pp16r.h; uses
// IgemmParams, M32Loader, lds_sw, wait_vm_c, store_partial, epi_pass, epi_rows_plain).
//
// Why (profiles/r04_ablation.txt): the ping-pong kernel (igemm_pp16.h, tiles 40 / 41) splits
// every K step into 4 phases of (load section | MFMA section), each closed by a barrier --
// 8 barriers and 4 lgkmcnt(0) drains per K step.  With the MFMAs and the DMA both removed
// that skeleton alone still took 65-70 us of the L0 conv's 105 us against 48 us of ideal
// MFMA time: the load section of a phase is as long as the partner's 20-MFMA section, so
// the matrix pipe idles whenever either runs long.
//
// What: the same tile, wave grid (8 waves = 2 row groups x 4 column waves, wave tile
// 128 x 16 TN), LDS-DMA loader and 2-slot ring of K-64 stages as tile 40, but no roles:
// every wave runs one K step as 16 MFMA groups g = (k32 half ks = g / 8, row tile b = g % 8)
// of TN MFMAs each, and issues its LDS reads INSIDE the MFMA stream, ahead of use:
//   * A row tile (ks, b) is read two groups before its group (a 4-entry register ring; the
//     last one, three: see below);
//   * the ks = 1 weight fragments during groups 2-6, the next step's ks = 0 weight fragments
//     and its first two A tiles during groups 14-15 (after the barrier, see below);
//   * the DMA pieces of the step after next go out one per group (groups 14, 15, 0, 1, ...).
// Two waves per SIMD run this same stream; while one waits on a fragment or holds its issue
// for a DMA piece, its partner's MFMAs keep the pipe fed.
// Synchronisation: ONE barrier per K step, after group 13 (X_kt):
//   before X_kt every wave waits lgkmcnt(0) (its last read of slot kt & 1, A(kt, 15), was
//   issued in group 12) and vmcnt(0) (its pieces of step kt + 1, all issued in groups
//   14-15 of step kt - 1 and 0..P-3 of step kt).
//   RAW: step kt + 1's slot is first read in group 14 of step kt, after X_kt.
//   WAR: the pieces of step kt + 2 overwrite slot kt & 1 from group 14 of step kt on, after
//   X_kt, which every wave passed only once its reads of that slot had completed; they are
//   read from group 14 of step kt + 1 on, after X_kt+1, before which every wave waited for them.
// Registers: accumulators 4 TN x 8 x 4 (160 at TN = 5), weight fragments 2 x 4 TN (both k32
// halves live across the step seam), A ring 16: ~230 with the loader state, under the 256 of
// two waves per SIMD.
#pragma once

namespace c2d {

#ifdef C2D_SP_STAMP
// Diagnostic build only (build.py --variant stamp --define C2D_SP_STAMP): s_memtime stamps of one
// workgroup's waves, 4 per K step, into a buffer nothing else reads (c2d_debug_sp_stamps copies it
// out).  The production library has no stamp code.
constexpr int kStampSteps = 64, kStampPer = 4 * kStampSteps + 4;
__device__ unsigned long long g_sp_stamps[8 * kStampPer];
#define C2D_STAMP(idx)                                                                             \
    do {                                                                                          \
        if (blockIdx.x == 77 && lane == 0 && (idx) < kStampPer)                                   \
            g_sp_stamps[wave * kStampPer + (idx)] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
#else
#define C2D_STAMP(idx) do {} while (0)
#endif

// STG: waves 4-7 (each the SIMD partner of wave w - 4) deal their pieces of step kt + 1 STG groups
// later than waves 0-3, so the two waves of a SIMD do not hold their issue for DMA pieces together
template <int TN, int KS, int STG>
__global__ void __launch_bounds__(512) igemm_sp_kernel(IgemmParams p) {
    constexpr int BK = 64, NW = 8, TMW = 8;
    constexpr int BM = 2 * TMW * 16, BN = 4 * TN * 16;
    constexpr int RB = 2 * BK, STAGE = (BM + BN) * RB;
    typedef M32Loader<BM, BN, BK, NW, KS, 0, true> Loader;
    constexpr int P = Loader::PMAX;
    static_assert(Loader::PMIN == P, "every wave deals the same pieces");
    static_assert(P >= 2 && P - 2 + STG <= 12, "pieces per wave per K step (all landed by X_kt)");
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

    C2D_STAMP(0);
    Loader ld;
    ld.init(p, m0, n0, wave, lane, kb);
    // fragment offsets: 16x16x32 operand = 16 rows (lane & 15) x 8 k (chunk lane >> 4) per k32
    const int fo0 = lds_sw<BK>(lane & 15, lane >> 4), fo1 = lds_sw<BK>(lane & 15, 4 + (lane >> 4));
    const int a_off0 = wr * TMW * 16 * RB + fo0, a_off1 = wr * TMW * 16 * RB + fo1;
    const int b_off0 = BM * RB + wc * TN * 16 * RB + fo0, b_off1 = BM * RB + wc * TN * 16 * RB + fo1;

    f32x4 acc[TN][TMW];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TMW; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

#define C2D_BAR() do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
#define C2D_LGKM0() __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14))
    // prologue: all of step kb, then pieces 0, 1 of step kb + 1 (the loop deals the rest in
    // its groups 0..P-3); wait for step kb only
    // (the loader position of step kt + 1, whose pieces 2.. step kt deals, is carried as two
    // ints and its descriptors rebuilt each step: a Stage carried across the loop's branches
    // became a scratch alloca)
    int tap1 = 0, cbase1 = 0;
    if (kb < ke) ld.issue(p, kb, smem + (kb & 1) * STAGE, wave);
    if (kb + 1 < ke) {
        tap1 = ld.tap;
        cbase1 = ld.cbase;
        const typename Loader::Stage s1 = ld.prep(p);
        ld.advance();
        ld.piece(s1, smem + ((kb + 1) & 1) * STAGE, wave, 0);
        ld.piece(s1, smem + ((kb + 1) & 1) * STAGE, wave, 1);
        wait_vm_c<2>();
    } else {
        wait_vm_c<0>();
    }
    C2D_BAR();

    C2D_STAMP(1);
    f16x8 fb0[TN], fb1[TN], fa[4];
    {
        const char* S = smem + (kb & 1) * STAGE;
#pragma unroll
        for (int t = 0; t < TN; ++t) fb0[t] = *reinterpret_cast<const f16x8*>(S + b_off0 + t * 16 * RB);
        fa[0] = *reinterpret_cast<const f16x8*>(S + a_off0);
        fa[1] = *reinterpret_cast<const f16x8*>(S + a_off0 + 16 * RB);
    }

    for (int kt = kb; kt < ke; ++kt) {
        const char* S = smem + (kt & 1) * STAGE;          // this step's slot
        const char* Sn = smem + ((kt + 1) & 1) * STAGE;   // the next step's (read after X_kt)
        char* Wn = smem + ((kt + 1) & 1) * STAGE;         // pieces 2.. of step kt + 1
        char* W2 = smem + (kt & 1) * STAGE;               // pieces 0, 1 of step kt + 2 (after X_kt)
        const bool nxt = kt + 1 < ke, nxt2 = kt + 2 < ke;
        const typename Loader::Stage st = ld.prep_at(p, tap1, cbase1);   // step kt + 1
        // the reads of the previous step's groups 14-15 (this step's first fragments) have had
        // 1.5 groups: an explicit wait here keeps the compiler from draining this group's own read
        C2D_LGKM0();
        C2D_STAMP(4 + 4 * (kt - kb));
        static_for<0, 16>([&](auto G) __attribute__((always_inline)) {
            constexpr int g = decltype(G)::value;
            constexpr int ks = g >> 3, b = g & 7;
            // ---- LDS reads ahead of use: A(g + 2) in group g, except that A(15) goes with A(14) in
            // group 12, so the lgkmcnt(0) before X_kt (after group 13) finds it landed
            auto read_a = [&](auto G2) __attribute__((always_inline)) {
                constexpr int g2 = decltype(G2)::value, ks2 = g2 >> 3, b2 = g2 & 7;
                fa[g2 & 3] = *reinterpret_cast<const f16x8*>(S + (ks2 ? a_off1 : a_off0) + b2 * 16 * RB);
            };
            if constexpr (g + 2 < 15) read_a(std::integral_constant<int, g + 2>{});
            if constexpr (g == 12) read_a(std::integral_constant<int, 15>{});
            if constexpr (g >= 2 && g < 2 + TN)
                fb1[g - 2] = *reinterpret_cast<const f16x8*>(S + b_off1 + (g - 2) * 16 * RB);
            // (unconditional: after the last step they read a stale slot and are never used, and
            // no branch hides them from the compiler's lgkmcnt counting)
            if constexpr (g == 14) {
#pragma unroll
                for (int t = 0; t < TN; ++t) fb0[t] = *reinterpret_cast<const f16x8*>(Sn + b_off0 + t * 16 * RB);
                fa[0] = *reinterpret_cast<const f16x8*>(Sn + a_off0);
            }
            if constexpr (g == 15) fa[1] = *reinterpret_cast<const f16x8*>(Sn + a_off0 + 16 * RB);
            // ---- MFMAs of this group (the DMA piece, if any, after the first)
            const f16x8 av = fa[g & 3];
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                if (C2D_ABL(p.abl, 2))   // timing ablation: fragments kept live, no MFMA
                    asm volatile("" :: "v"(ks ? fb1[a] : fb0[a]), "v"(av));
                else
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ks ? fb1[a] : fb0[a], av, acc[a][b], 0, 0, 0);
                if (a == 0 && !C2D_ABL(p.abl, 1)) {
                    if constexpr (g < P - 2) {
                        if (nxt && (STG == 0 || wr == 0)) ld.piece(st, Wn, wave, g + 2);
                    }
                    if constexpr (STG > 0 && g >= STG && g - STG < P - 2) {
                        if (nxt && wr == 1) ld.piece(st, Wn, wave, g - STG + 2);
                    }
                    if constexpr (g == 14) {
                        if (nxt2) {   // step kt + 2: pieces 0 and 1 now, the rest in step kt + 1
                            tap1 = ld.tap;
                            cbase1 = ld.cbase;
                            ld.advance();
                            ld.piece(ld.prep_at(p, tap1, cbase1), W2, wave, 0);
                        }
                    }
                    if constexpr (g == 15) {
                        if (nxt2) ld.piece(ld.prep_at(p, tap1, cbase1), W2, wave, 1);
                    }
                }
            }
            if constexpr (g == 13) {   // X_kt: slot kt & 1 fully read, slot (kt + 1) & 1 landed
                C2D_STAMP(5 + 4 * (kt - kb));
                wait_vm_c<0>();
                C2D_LGKM0();
                C2D_STAMP(6 + 4 * (kt - kb));
                C2D_BAR();
                C2D_STAMP(7 + 4 * (kt - kb));
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    }
#undef C2D_BAR
#undef C2D_LGKM0
    C2D_STAMP(2);

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
    // LDS-staged epilogue, as igemm_pp16.h (every wave's reads of the ring are complete:
    // the barrier below follows the last K step's MFMAs)
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
    } else {
        constexpr int PITCHB = BN + 4;
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
    C2D_STAMP(3);
}

template <int TN, int KS, int STG>
static void launch_sp(const IgemmParams& p, hipStream_t s) {
    constexpr int ring = 2 * (256 + 4 * TN * 16) * 128;
    constexpr int epi_wg = 64 * (4 * TN * 16 + 4) * 4, epi_wv = 8 * 32 * (TN * 16 + 4) * 4;   // epilogue images
    constexpr int epi = epi_wg > epi_wv ? epi_wg : epi_wv;
    constexpr int smem = ring > epi ? ring : epi;
    static_assert(smem <= 160 * 1024, "LDS ring / epilogue image too large");
    ensure_lds<igemm_sp_kernel<TN, KS, STG>>(smem);
    hipLaunchKernelGGL((igemm_sp_kernel<TN, KS, STG>), dim3(p.gx * p.gy * p.ksplit), dim3(512), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

template <int TN, int STG>
static void run_sp(IgemmParams& p, int ksize, int cout, hipStream_t s) {
    constexpr int BM = 256, BN = 4 * TN * 16;
    p.gx = (cout + BN - 1) / BN;
    p.gy = (p.M + BM - 1) / BM;
    if (ksize == 1) launch_sp<TN, 1, STG>(p, s);
    else launch_sp<TN, 3, STG>(p, s);
}

}  // namespace c2d
