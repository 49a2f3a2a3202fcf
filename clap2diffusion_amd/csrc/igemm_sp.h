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
constexpr int kStampSteps = 64, kStampPer = 6 * kStampSteps + 4;
__device__ unsigned long long g_sp_stamps[8 * kStampPer];
#define C2D_STAMP(idx)                                                                             \
    do {                                                                                          \
        if (blockIdx.x == 77 && lane == 0 && (idx) < kStampPer)                                   \
            g_sp_stamps[wave * kStampPer + (idx)] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
#else
#define C2D_STAMP(idx) do {} while (0)
#endif

#ifndef C2D_SP_ABL
#define C2D_SP_ABL 0   // diagnostic variant builds only (wrong results): 1 = no DMA after the prologue,
                       // 2 = no A pieces, 4 = no B pieces
#endif

// LDS-DMA staging of one K-64 step of the 256 x BN tile (A = im2col rows, B = packed weight
// rows, the igemm_dma_kernel / M32Loader addressing and lane-linear XOR-swizzled image) dealt by
// FOUR of the eight waves: loader wave d (0..3) issues the 1-KiB pieces of LDS slots d + 4 k.
// Why four: a DMA piece holds its wave's issue until the CU's vector-memory path takes it (the
// path moves ~64 B per clock, so a K step's 72 pieces keep it busy ~1150 cycles); with every
// wave dealing, the two waves of a SIMD stalled together and the matrix pipe idled (timeline
// stamps: ~1100 of ~4600 cycles per K step).  Waves 0-3 (the SIMD partners of 4-7) deal them
// all, so on every SIMD one wave keeps issuing MFMAs while the other waits on the DMA path.
// Per lane: the window pixel of each of its 8 A rows, their 3x3 tap masks packed 3 per register,
// one weight-row offset (the 10 B slots of a loader wave are 32 rows apart).
template <int BN, int KS>
struct SpLoader {
    static constexpr int BM = 256, BK = 64, RB = 2 * BK;
    static constexpr int NA = BM / 8 / 4, NB = BN / 8 / 4;   // A / B pieces per loader wave
    static constexpr int P = NA + NB;                         // pieces per loader wave per K step
    static_assert(BN % 32 == 0, "B rows split over four loader waves");
    int a_pix[NA];
    unsigned a_mpk[3];        // 9-bit tap masks of A rows k, 3 per register (k / 3, bits 9 (k % 3))
    unsigned b_off0;          // byte offset of this lane's row of B slot 0 (kOOB past cout)
    int b_row0, ch;           // weight row of B slot 0; the swizzled channel chunk (every slot the same)
    unsigned bytes0, bytes1, wbytes;
    const char *u_src0, *u_src1, *u_wt;
    int pshift, tap, cbase, cin_, cout_, kpad2;
    bool two, ctail, cmajor;

    __device__ __forceinline__ void init(const IgemmParams& p, int m0, int n0, int d, int lane, int kb) {
        const int lrow = lane >> 3, lchunk = lane & 7;
        const int hw = p.oh * p.ow;
        two = p.c1 > 0;
        pshift = KS == 3 ? p.w + 1 : 0;
        // (row >> 1) & 7 of row (d + 4 k) * 8 + lrow is (4 d + (lrow >> 1)) & 7 for every k
        ch = (lchunk ^ ((4 * d + (lrow >> 1)) & 7)) * 8;
        a_mpk[0] = a_mpk[1] = a_mpk[2] = 0;
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const int m = m0 + (d + 4 * k) * 8 + lrow;
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
                        if (iy0 + ky >= 0 && iy0 + ky < p.h && ix0 + kx >= 0 && ix0 + kx < p.w)
                            mask |= 1u << (ky * KS + kx);
            }
            a_pix[k] = (nn * p.h + iy0) * p.w + ix0 + pshift;
            a_mpk[k / 3] |= mask << (9 * (k % 3));
        }
        b_row0 = n0 + d * 8 + lrow;
        kpad2 = 2 * p.kpad;
        b_off0 = (unsigned)(b_row0 * kpad2 + 2 * ch);
        cout_ = p.cout;
        const size_t npix = (size_t)p.n * p.h * p.w;
        bytes0 = (unsigned)(npix * p.c0 * 2);
        bytes1 = (unsigned)(npix * p.c1 * 2);
        wbytes = (unsigned)((size_t)p.cout * p.kpad * 2);
        ctail = (p.cin % BK) != 0;
        cin_ = p.cin;
        cmajor = p.cmajor != 0;
        u_src0 = uniform_ptr(p.src0);
        u_src1 = uniform_ptr(p.src1);
        u_wt = uniform_ptr(p.wt);
        cbase = kb * BK;
        tap = 0;
        if (KS == 3) {
            if (p.cmajor) { tap = kb % 9; cbase = (kb / 9) * BK; }
            else { tap = cbase / p.cin; cbase -= tap * p.cin; }
        }
    }
    struct Stage {
        __amdgpu_buffer_rsrc_t ra, rb;
        int cs, lim, tap;
    };
    __device__ __forceinline__ Stage prep_at(const IgemmParams& p, int tp, int cb) const {
        Stage st;
        const int k0 = tp * p.cin + cb;
        const int ky = tp / 3, kx = tp - (tp / 3) * 3;
        const bool use1 = two && cb >= p.c0;
        st.cs = use1 ? p.c1 : p.c0;
        const unsigned sterm = 2u * (unsigned)((KS == 3 ? (ky * p.w + kx) * st.cs : 0) + (use1 ? cb - p.c0 : cb));
        const char* sb = use1 ? u_src1 : u_src0;
        const unsigned bias = 2u * (unsigned)(pshift * st.cs);
        const unsigned sbytes = use1 ? bytes1 : bytes0;
        st.ra = make_rsrc(sb + sterm - bias, sbytes + bias - sterm);
        st.rb = make_rsrc(u_wt + 2 * k0, wbytes - 2 * k0);
        st.lim = p.cin - cb;
        st.tap = tp;
        return st;
    }
    // piece q (< P; A slots first) of loader wave d into the stage image at lds
    __device__ __forceinline__ void piece(const Stage& st, char* lds, int d, int q) const {
        if ((C2D_SP_ABL & 2) && q < NA) return;    // diagnostic variants: no A / no B pieces
        if ((C2D_SP_ABL & 4) && q >= NA) return;
        if (q < NA) {
            unsigned ok = (a_mpk[q / 3] >> (9 * (q % 3) + st.tap)) & 1u;
            if (ctail) ok &= (unsigned)(ch < st.lim);
            // pixel x channel stride < 2^31 bytes (dma_eligible), both factors < 2^24
            const unsigned off = (__umul24((unsigned)a_pix[q], (unsigned)st.cs) + (unsigned)ch) * 2u;
            dma_piece(st.ra, lds + (d + 4 * q) * 1024, off | ((ok - 1u) & kOOB));
        } else {
            const int k = q - NA;
            const bool ok = (d + 4 * k) * 8 < BN && b_row0 + 32 * k < cout_;
            dma_piece(st.rb, lds + BM * RB + (d + 4 * k) * 1024, ok ? b_off0 + (unsigned)(k * 32 * kpad2) : kOOB);
        }
    }
    __device__ __forceinline__ void advance() {
        if (KS == 3 && cmajor) {
            if (++tap == 9) { tap = 0; cbase += BK; }
        } else {
            cbase += BK;
            if (KS == 3 && cbase >= cin_) { cbase = 0; ++tap; }
        }
    }
};


// The output of a 256 x 16 TN tile held as 8 waves' 128 x 16 TN accumulators (waves 2 x 4):
// split-K partials, or the LDS-staged epilogue of igemm_pp16.h (bias / act / GEGLU / temb /
// residual; every wave's ring reads must be complete -- its barrier is the first thing here)
template <int TN>
__device__ __forceinline__ void sp_epilogue(const IgemmParams& p, f32x4 (&acc)[TN][8], int m0, int n0, int slice,
                                            int wave, int lane, int tid, char* smem) {
    constexpr int TMW = 8, BN = 4 * TN * 16;
    const int wr = wave >> 2, wc = wave & 3;
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
}

template <int TN, int KS>
__global__ void __launch_bounds__(512) igemm_sp_kernel(IgemmParams p) {
    constexpr int BK = 64, NW = 8, TMW = 8;
    constexpr int BM = 2 * TMW * 16, BN = 4 * TN * 16;
    constexpr int RB = 2 * BK, STAGE = (BM + BN) * RB;
    typedef SpLoader<BN, KS> Loader;
    constexpr int P = Loader::P;   // pieces per loader wave per K step: 4 after X2, 2 per group in groups 0..
    static_assert(P >= 6 && P <= 18, "pieces per loader wave per K step");
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
    const int dw = wave & 3;           // loader wave index (waves 0-3 deal the DMA)
    const bool loader = wave < 4;
    ld.init(p, m0, n0, dw, lane, kb);
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
#define C2D_LGKM(N) __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | ((N) << 8) | (3 << 14))
    // prologue: all of step kb, then piece 0 of step kb + 1 (the loop deals the rest in its
    // groups 0-4); wait for step kb only.  The loader position of the step whose later pieces a
    // step deals is carried as two ints and its descriptors rebuilt there (a Stage carried
    // across the loop's branches became a scratch alloca).
    int tap1 = 0, cbase1 = 0;
    if (loader) {
        if (kb < ke) {
            const typename Loader::Stage s0 = ld.prep_at(p, ld.tap, ld.cbase);
            ld.advance();
#pragma unroll
            for (int q = 0; q < P; ++q) ld.piece(s0, smem + (kb & 1) * STAGE, dw, q);
        }
        if (kb + 1 < ke) {
            tap1 = ld.tap;
            cbase1 = ld.cbase;
            const typename Loader::Stage s1 = ld.prep_at(p, tap1, cbase1);
            ld.advance();
#pragma unroll
            for (int q = 0; q < 4; ++q) ld.piece(s1, smem + ((kb + 1) & 1) * STAGE, dw, q);
            wait_vm_c<4>();
        } else {
            wait_vm_c<0>();
        }
    } else if (kb + 1 < ke) {   // keep the non-loader waves' loader position in step (unused)
        tap1 = 0;
    }
    C2D_BAR();

    C2D_STAMP(1);
#ifdef C2D_SP_PRIO
    if (!loader) __builtin_amdgcn_s_setprio(C2D_SP_PRIO);   // diagnostic variant: the MFMA-only waves first
#endif
    f16x8 fb0[TN], fb1[TN], fa[4];
    {
        const char* S = smem + (kb & 1) * STAGE;
#pragma unroll
        for (int t = 0; t < TN; ++t) fb0[t] = *reinterpret_cast<const f16x8*>(S + b_off0 + t * 16 * RB);
#pragma unroll
        for (int t = 0; t < 3; ++t) fa[t] = *reinterpret_cast<const f16x8*>(S + a_off0 + t * 16 * RB);
    }

    for (int kt = kb; kt < ke; ++kt) {
        const char* S = smem + (kt & 1) * STAGE;          // this step's slot
        const char* Sn = smem + ((kt + 1) & 1) * STAGE;   // the next step's (read after X1)
        char* Wn = smem + ((kt + 1) & 1) * STAGE;         // pieces 4.. of step kt + 1 (groups 0..)
        char* W2 = smem + (kt & 1) * STAGE;               // pieces 0-3 of step kt + 2 (groups 14-15, after X2)
        const bool nxt = kt + 1 < ke, nxt2 = kt + 2 < ke;
        const typename Loader::Stage st = ld.prep_at(p, tap1, cbase1);   // step kt + 1
        // the previous step's reads of this step's first fragments (groups 11-15) retired here,
        // so the counts the compiler derives inside the step start from zero (it cannot follow
        // them across the loop edge and would otherwise drain group 0's own read)
        C2D_LGKM(0);
        C2D_STAMP(4 + 6 * (kt - kb));
        static_for<0, 16>([&](auto G) __attribute__((always_inline)) {
            constexpr int g = decltype(G)::value;
            constexpr int ks = g >> 3, b = g & 7;
            // ---- LDS reads ahead of use (after the step's last read of slot kt & 1, A(15) in group
            // 12, only slot (kt + 1) & 1, behind X1; unconditional: after the last step they read a
            // stale slot and are never used, and no branch hides them from the lgkmcnt counting)
            if constexpr (g + 3 < 16) {
                constexpr int g3 = g + 3, ks3 = g3 >> 3, b3 = g3 & 7;
                fa[g3 & 3] = *reinterpret_cast<const f16x8*>(S + (ks3 ? a_off1 : a_off0) + b3 * 16 * RB);
            } else {
                constexpr int g3 = g + 3 - 16;   // next step's A(0..2), ks = 0
                fa[g3 & 3] = *reinterpret_cast<const f16x8*>(Sn + a_off0 + g3 * 16 * RB);
            }
            if constexpr (g >= 1 && g <= TN) fb1[g - 1] = *reinterpret_cast<const f16x8*>(S + b_off1 + (g - 1) * 16 * RB);
            if constexpr (g >= 11 && g <= 14) {   // the next step's ks = 0 weight fragments: 2, 1, 1, 1
                constexpr int t0 = g == 11 ? 0 : g - 10, t1 = g == 11 ? 2 : g - 9;
#pragma unroll
                for (int t = t0; t < t1 && t < TN; ++t) fb0[t] = *reinterpret_cast<const f16x8*>(Sn + b_off0 + t * 16 * RB);
            }
            // ---- MFMAs of this group (its DMA pieces, if any, after the first)
            const f16x8 av = fa[g & 3];
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ks ? fb1[a] : fb0[a], av, acc[a][b], 0, 0, 0);
                if (a == 0 && !(C2D_SP_ABL & 1)) {
                    // loader waves only; step kt + 1: pieces 4.. (2 per group; 0-3 went out in groups
                    // 14-15 of step kt - 1)
                    if constexpr (2 * g + 4 < P && g < 8) {
                        if (loader && nxt) {
                            ld.piece(st, Wn, dw, 2 * g + 4);
                            if constexpr (2 * g + 5 < P) ld.piece(st, Wn, dw, 2 * g + 5);
                        }
                    }
                    // step kt + 2: pieces 0-3, two per group after X2
                    if constexpr (g == 14) {
                        if (loader && nxt2) {
                            tap1 = ld.tap;
                            cbase1 = ld.cbase;
                            ld.advance();
                            const typename Loader::Stage s2 = ld.prep_at(p, tap1, cbase1);
                            ld.piece(s2, W2, dw, 0);
                            ld.piece(s2, W2, dw, 1);
                        }
                    }
                    if constexpr (g == 15) {
                        if (loader && nxt2) {
                            const typename Loader::Stage s2 = ld.prep_at(p, tap1, cbase1);
                            ld.piece(s2, W2, dw, 2);
                            ld.piece(s2, W2, dw, 3);
                        }
                    }
                }
            }
            if constexpr (g == 10) {   // X1: every wave's pieces of step kt + 1 landed (RAW of its slot)
                C2D_STAMP(5 + 6 * (kt - kb));
                wait_vm_c<0>();
                C2D_BAR();
                C2D_STAMP(6 + 6 * (kt - kb));
            }
            if constexpr (g == 13) {   // X2: every wave's reads of slot kt & 1 done (WAR for step kt + 2)
                // >= 2 reads of the next slot (groups 12-13) were issued after A(15): lgkmcnt(2)
                // retires A(15) and everything before it
                C2D_LGKM(2);
                C2D_BAR();
                C2D_STAMP(7 + 6 * (kt - kb));
            }
            if constexpr (g == 14) C2D_STAMP(8 + 6 * (kt - kb));
            if constexpr (g == 15) C2D_STAMP(9 + 6 * (kt - kb));
            __builtin_amdgcn_sched_barrier(0);
        });
    }
#undef C2D_BAR
#undef C2D_LGKM
    C2D_STAMP(2);

    sp_epilogue<TN>(p, acc, m0, n0, slice, wave, lane, tid, smem);
    C2D_STAMP(3);
}

template <int TN, int KS>
static void launch_sp(const IgemmParams& p, hipStream_t s) {
    constexpr int ring = 2 * (256 + 4 * TN * 16) * 128;
    constexpr int epi_wg = 64 * (4 * TN * 16 + 4) * 4, epi_wv = 8 * 32 * (TN * 16 + 4) * 4;   // epilogue images
    constexpr int epi = epi_wg > epi_wv ? epi_wg : epi_wv;
    constexpr int smem = ring > epi ? ring : epi;
    static_assert(smem <= 160 * 1024, "LDS ring / epilogue image too large");
    ensure_lds<igemm_sp_kernel<TN, KS>>(smem);
    hipLaunchKernelGGL((igemm_sp_kernel<TN, KS>), dim3(p.gx * p.gy * p.ksplit), dim3(512), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

template <int TN>
static void run_sp(IgemmParams& p, int ksize, int cout, hipStream_t s) {
    constexpr int BM = 256, BN = 4 * TN * 16;
    p.gx = (cout + BN - 1) / BN;
    p.gy = (p.M + BM - 1) / BM;
    if (ksize == 1) launch_sp<TN, 1>(p, s);
    else launch_sp<TN, 3>(p, s);
}

}  // namespace c2d
