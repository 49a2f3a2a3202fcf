// Row-ring ping-pong 3x3 conv (tiles 42 / 43 / 44; included by igemm.hip after igemm_pps.h; uses
// IgemmParams, lds_sw, wait_vm_c, make_rsrc, kOOB, store_partial, epi_pass, epi_rows_plain).
//
// Why: the one-shot ping-pong conv (igemm_pp16.h, tile 40) stages, per 64-deep K step, a
// 256-row A tile (one 3x3 tap of one 64-channel block) and a 320-row weight tile: 72 LDS-DMA
// pieces of 1 KiB, 9 per wave, each holding its wave's issue for 60-185 cycles -- the load
// section of every phase is as long as the partner's MFMA section (MFMA busy 0.48); the im2col
// A pieces cost ~900 cycles of issue per K step against ~200 for the weights
// (profiles/r05_sp_timeline.txt).  The nine taps of one channel block re-read, from L2, nine
// shifted copies of the same few image rows.
//
// What: the input is the zero-bordered layout [n][h + 2][w + 2][c] (c2d_conv_desc::src_pad,
// written by c2d_groupnorm_pad), so every tap of every output pixel is in bounds: the conv is a
// "valid" 3x3 over the padded image and needs no masks.  An output tile of BM = 2 TMW 16 rows
// is R = BM / W whole image rows of one image; the 9 K steps of a channel block read RB = R + 2
// padded image rows, staged ONCE per channel block into a ring of NS row slots of SP = 8 PPR
// LDS rows (128 B: one padded pixel x 64 channels; PPR pieces of 8 pixels per row, the last
// piece over-reads into the next padded row, never read), and every tap's A fragment is a
// row-shifted read of a slot: per channel block RB x PPR A pieces instead of 9 x BM / 8.
//   tile 42: W = 64, BM = 256 (R = 4, RB = 6, NS = 8, SP = 72)   c3's level-0 ResnetBlock2D convs
//   tile 43: W = 32, BM = 128 (R = 4, RB = 6, NS = 8, SP = 40)   level 1: 256 tiles at N = 16, no split
//   tile 44: W = 16, BM = 128 (R = 8, RB = 10, NS = 16, SP = 20)  level 2
// Row schedule (RrSched): row j of channel block c sits in slot (RB c + j) mod NS; the rows a
// ky phase (3 K steps) issues are listed per RB, each into the slot of a row whose last tap ran
// in an earlier ky phase (row j is read by the taps ky in [j - R + 1, j]) and each landed (vmcnt(0)
// + barrier) before its first tap.  A K step issues pieces q = 3 wave + kx of its phase's list.
// Bank swizzle of the A slots: 16-B chunk c of LDS row r sits at slot c ^ (r & 6).  Found by
// exhaustive search over the ds_read_b128 lane groups (MI355X_MICROARCH.md §LDS): conflict-free
// for a 16-row fragment starting at ANY row and both k32 halves, so slot pitches need only be
// multiples of 8 (the DMA piece: then chunk ^ (r & 6) = chunk ^ (lane row & 6) per lane) and
// 16-row tiles at x0 = 16 t are ds_read immediates.  (Round 4's rr_swz table covered row shifts
// 0..2 only, which forced 16-row-aligned slots of 80 rows.)
// LDS: the A slots + a 2-slot weight ring (2 x 40 KiB at BN = 320).  The MFMA / phase / barrier
// structure is igemm_pp16.h's (PH = 4 phases per K step (k32 half, row half) at TMW = 8, PH = 2
// (k32 half) at TMW = 4; the two row groups one barrier apart; next-step weight pieces dealt
// in phases 0..PH-2, every own piece waited in the last phase).  Split-K slices own whole
// channel blocks.
#pragma once

namespace c2d {

// steady-state row schedule of one channel block c: per ky phase, the rows (db, j) it issues
// (db = 0: block c's own late rows, needed from a later ky phase of c; db = 1: block c + 1's,
// issued only when c + 1 is in the slice), and the rows of block 0 the prologue stages
// (entry e of ky phase ky: code db << 4 | j; n: entries per phase)
template <int RB> struct RrSched;
template <> struct RrSched<6> {    // NS = 8: (c,4),(c,5) | (c+1,0),(c+1,2) | (c+1,1),(c+1,3)
    static constexpr int NS = 8, PRO = 4, NMAX = 2;
    __host__ __device__ static constexpr int n(int) { return 2; }
    __host__ __device__ static constexpr int code(int ky, int e) {
        return ky == 0 ? (e == 0 ? 0x04 : 0x05) : ky == 1 ? (e == 0 ? 0x10 : 0x12) : (e == 0 ? 0x11 : 0x13);
    }
};
template <> struct RrSched<10> {   // NS = 16: (c,8),(c,9),(c+1,0),(c+1,1) | (c+1,2),(c+1,3),(c+1,6) | (c+1,4),(c+1,5),(c+1,7)
    static constexpr int NS = 16, PRO = 8, NMAX = 4;
    __host__ __device__ static constexpr int n(int ky) { return ky == 0 ? 4 : 3; }
    __host__ __device__ static constexpr int code(int ky, int e) {
        constexpr unsigned long long T0 = 0x1110'0908ull, T1 = 0x0016'1312ull, T2 = 0x0017'1514ull;   // bytes e = 0..3
        return (int)(((ky == 0 ? T0 : ky == 1 ? T1 : T2) >> (8 * e)) & 0xffu);
    }
};

#ifndef C2D_PP16R_RRSWZ
#define C2D_PP16R_RRSWZ 0   // 1: tile 42 with round 4's layout (80-row slots, rr_swz; A/B builds)
#endif
// Round 4's bank swizzle of tile 42 (A/B builds only): conflict-free for row shifts 0..2 only,
// repeating every 16 rows, so slots were 80 rows apart.  f = {0,0,1,1,2,2,4,4, 5,5,6,6,2,2,6,6}
__host__ __device__ constexpr int rr_swz(int r) {
    constexpr unsigned long long F = 0ull | (0ull << 3) | (1ull << 6) | (1ull << 9) | (2ull << 12) | (2ull << 15) |
                                     (4ull << 18) | (4ull << 21) | (5ull << 24) | (5ull << 27) | (6ull << 30) |
                                     (6ull << 33) | (2ull << 36) | (2ull << 39) | (6ull << 42) | (6ull << 45);
    return (int)((F >> (3 * r)) & 7ull);
}

template <int W, int BM_> struct RrGeo {
    static constexpr int BM = BM_, R = BM / W, RB = R + 2;
    static constexpr int PPR = (W + 2 + 7) / 8;                 // pieces per padded row
    // LDS rows per slot: 8 PPR, or 20 at W = 16 (18 pixels: the slot ring of 16 fits beside a 3-slot
    // weight ring).  There the last piece of a row loads its 2 pixels with lanes 0-15 only (LASTL),
    // and slots start at rows = 4 mod 8 on odd slots, whose chunk swizzle is then (r + 4) & 6 (PAR)
    static constexpr bool RR = C2D_PP16R_RRSWZ && W == 64;
    static constexpr int SP = RR ? 80 : W == 16 ? 20 : PPR * 8;
    __host__ __device__ static constexpr int swz(int r) { return RR ? rr_swz(r & 15) : (r & 6); }
    static constexpr bool PAR = (SP % 8) != 0;
    static constexpr int LASTL = SP < PPR * 8 ? ((W + 2) - 8 * (PPR - 1)) * 8 : 64;
    static_assert(SP % 4 == 0 && SP >= W + 2, "slot pitch");
    typedef RrSched<RB> S;
    static constexpr int NS = S::NS;
    static constexpr int A_BYTES = NS * SP * 128;
    static_assert(BM % W == 0 && W % 16 == 0, "whole image rows per tile, whole 16-row fragments per row");
    static_assert(S::n(0) * PPR <= 24 && S::n(1) * PPR <= 24 && S::n(2) * PPR <= 24, "pieces per ky phase");
};

// PH phases per K step: 4 = (k32 half, row half), 20-MFMA sections (TMW = 8); 2 = k32 half
// (TMW = 4: one row half; TMW = 8: 40-MFMA sections, every weight piece dealt in phase 0)
// NB: weight ring slots.  2: the pieces of K step kt + 1 are dealt in step kt and waited at its end.
// 3 (tile 43): the pieces of step kt + 2, dealt over both phases and waited one step later
// (vmcnt(NBP): everything older than this step's weight pieces), so no phase's load section
// carries all NBP pieces of a step (the 2-phase form dealt them all in phase 0)
// NRG: row groups of the 8 waves (2: 2 x 4 column waves, the ping-pong layout of igemm_pp16.h;
// 4: 4 x 2).  Waves 0-3 and 4-7 are the two stagger groups either way (one wave of each per SIMD),
// group 1 one barrier behind group 0.  A 128 x 160 width-16 tile on the 4 x 2 layout (TMW = 2,
// 10-MFMA phases; round 6, built and measured: profiles/r06_rr_sweep45_b*.txt) ran c3's level-2
// 1280 -> 1280 conv unsplit at 175.5 us against 126.8 for (40, 4) and lost at every split: only
// NRG = 2 is instantiated.
template <int TN, int PH, int W, int TMW, int NB = 2, int NRG = 2>
__global__ void __launch_bounds__(512) igemm_pp16r_kernel(IgemmParams p) {
    constexpr int NCW = 8 / NRG;                    // column waves
    typedef RrGeo<W, NRG * TMW * 16> G;
    typedef typename G::S S;
    static_assert(PH == 2 || PH == 4, "pp16r phases per K step");
    static_assert(NB == 2 || (NB == 3 && PH == 2), "weight ring depth");
    static_assert(TMW == 8 || (TMW <= 4 && PH == 2), "row halves per phase");
    static_assert(NRG == 2 || NRG == 4, "row groups");
    constexpr int BK = 64, NW = 8;
    constexpr int RT = PH == 4 ? 4 : TMW;           // 16-row tiles per phase
    constexpr int BM = G::BM, BN = NCW * TN * 16;
    constexpr int RB = 2 * BK;                    // bytes per LDS row
    constexpr int SBYTES = G::SP * RB;            // bytes per row slot
    constexpr int A_BYTES = G::A_BYTES;
    constexpr int BSTAGE = BN * RB;
    constexpr int NPB = BN / 8;                   // weight pieces per K step
    constexpr int NBP = (NPB + NW - 1) / NW;      // ... per wave (the first NPB % NW waves one more)
    constexpr int PPR = G::PPR, NS = G::NS, ROWB = G::RB;
    static_assert(BN % 8 == 0, "whole weight pieces");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave / NCW, wc = wave - (wave / NCW) * NCW, sg = wave >> 2;
    const int nbp = (NPB - wave + NW - 1) / NW;   // this wave's weight pieces per K step
    const int l15 = lane & 15, lg = lane >> 4;
    const int lrow = lane >> 3, lchunk = lane & 7;
    const int bid = xcd_remap(blockIdx.x, p.gx * p.gy * p.ksplit);
    const int tile = bid / p.ksplit, slice = bid - tile * p.ksplit;
    const int mt = tile / p.gx, nt = tile - mt * p.gx;
    const int m0 = mt * BM, n0 = nt * BN;
    const int cin = p.cin;
    const int ncb_all = cin / BK, cbs = p.nkt / 9;
    const int cb0 = slice * cbs, ncb = min(ncb_all, cb0 + cbs) - cb0;
    // output tile = R whole image rows of image nimg starting at row y0 (host: ow = W, oh * ow % BM == 0)
    const int hw = p.oh * p.ow;
    const int nimg = m0 / hw, y0 = (m0 - nimg * hw) / p.ow;
    const int prow0 = (nimg * p.h + y0) * p.w;    // padded pixel index of relative row j = 0
    const unsigned a_img = 2u * (unsigned)(prow0 * cin + cb0 * BK), a_rowb = 2u * (unsigned)(p.w * cin);

    const char* u_src = uniform_ptr(p.src0);
    const char* u_wt = uniform_ptr(p.wt);
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(u_src, (unsigned)((size_t)p.n * p.h * p.w * cin * 2));
    const unsigned wbytes = (unsigned)((size_t)p.cout * p.kpad * 2);

    // A piece lane offset: pixel lrow of the piece, logical chunk lchunk ^ (lrow & 6) (pieces start
    // at LDS rows that are multiples of 8, so the slot swizzle is the same for every piece)
    // (RR: rows 8 k + lrow repeat every 16, so the piece's parity picks the half)
    const unsigned a_lo0 = (unsigned)(2 * (lrow * cin + ((lchunk ^ G::swz(lrow)) << 3)));
    const unsigned a_lo1 = (G::PAR || G::RR) ? (unsigned)(2 * (lrow * cin + ((lchunk ^ G::swz(lrow + (G::RR ? 8 : 4))) << 3)))
                                             : a_lo0;
    // weight rows of this wave's pieces (the M32Loader B addressing)
    unsigned b_off[NBP];
#pragma unroll
    for (int i = 0; i < NBP; ++i) {
        const int row = (wave + i * NW) * 8 + lrow;
        const int j = n0 + row;
        b_off[i] = j < p.cout ? (unsigned)(2 * (j * p.kpad + ((lchunk ^ ((row >> 1) & 7)) << 3))) : kOOB;
    }
    const int fo0 = lds_sw<BK>(l15, lg), fo1 = lds_sw<BK>(l15, 4 + lg);

    // one A piece: padded pixels 8k .. 8k + 7 of relative row j of channel block cr (relative)
    auto a_piece = [&](int cr, int j, int k) __attribute__((always_inline)) {
        const int s = (int)((unsigned)(ROWB * cr + j) % (unsigned)NS);
        const unsigned soff = a_img + (unsigned)j * a_rowb + 2u * (unsigned)(8 * k * cin + cr * BK);
        const unsigned lo = ((G::PAR && (s & 1)) || (G::RR && (k & 1))) ? a_lo1 : a_lo0;
        if (G::LASTL < 64 && k == PPR - 1) {
            if (lane < G::LASTL)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lptr_t)(smem + s * SBYTES + k * 1024), 16, lo, (int)soff, 0, 0);
        } else {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lptr_t)(smem + s * SBYTES + k * 1024), 16, lo, (int)soff, 0, 0);
        }
    };
    // weight piece i of K step (cr, tap) into ring slot bs (i < nbp)
    auto b_piece = [&](int cr, int tap, int bs, int i) __attribute__((always_inline)) {
        if (NPB % NW != 0 && i >= nbp) return;
        const int k0 = tap * cin + (cb0 + cr) * BK;
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(u_wt + 2 * k0, wbytes - 2 * k0);
        dma_piece(rb, smem + A_BYTES + bs * BSTAGE + (wave + i * NW) * 1024, b_off[i]);
    };
    // piece q of ky phase `ky` of channel block cr (the phase's rows in schedule order)
    auto sched_piece = [&](int cr, int ky, int q, bool more) __attribute__((always_inline)) {
        const int e = q / PPR, k = q - e * PPR;
        if (e >= S::n(ky)) return;
        const int code = S::code(ky, e), dbv = code >> 4;
        if (dbv && !more) return;
        a_piece(cr + dbv, code & 15, k);
    };

    f32x4 acc[TN][TMW];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TMW; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

#define C2D_BAR() do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
    // prologue: rows 0 .. PRO-1 of the first channel block and the weights of step 0
    if (ncb > 0) {
        for (int q = wave; q < S::PRO * PPR; q += NW) a_piece(0, q / PPR, q - (q / PPR) * PPR);
#pragma unroll
        for (int i = 0; i < NBP; ++i) b_piece(0, 0, 0, i);
        if (NB == 3 && 9 * ncb > 1) {
#pragma unroll
            for (int i = 0; i < NBP; ++i) b_piece(0, 1, 1, i);
        }
    }
    wait_vm_c<0>();
    C2D_BAR();
    if (sg) C2D_BAR();   // group 1 runs one barrier behind group 0

    f16x8 fa[RT], fb[TN];
    const int nsteps = 9 * ncb;
    int bs = 0;                                         // weight ring slot of this step
    for (int kt = 0; kt < nsteps; ++kt) {
        const int cr = kt / 9, tap = kt - cr * 9, ky = tap / 3, kx = tap - ky * 3;
        const bool more = cr + 1 < ncb;
        const bool nxt = kt + 1 < nsteps;
        // the weight pieces dealt in this step: step kt + NB - 1 into ring slot bw
        const int kd = kt + NB - 1;
        const bool bdeal = kd < nsteps;
        const int ncr = kd / 9, ntap = kd - (kd / 9) * 9;
        const int bw = NB == 2 ? (bs ^ 1) : (bs == 0 ? 2 : bs - 1);
        const char* SB = smem + A_BYTES + bs * BSTAGE + wc * TN * 16 * RB;
        // A fragment rows: LDS row kx + l15 (+ x0) of the slot of image row ir + ky of block cr
        const int ar = l15 + kx;
        const int alane = ar * RB + (((lg) ^ G::swz(ar)) << 4);   // k32 half 0; half 1: chunk bit 2 flipped
        const int alane1 = G::PAR ? ar * RB + (((lg) ^ G::swz(ar + 4)) << 4) : alane;   // odd slots (PAR)
        const int sbase = ROWB * cr + ky;
#pragma unroll
        for (int qq = 0; qq < PH; ++qq) {
            const int ks = PH == 4 ? qq >> 1 : qq, rh = PH == 4 ? qq & 1 : 0;
            // ---- load section
            if (rh == 0) {
#pragma unroll
                for (int t = 0; t < TN; ++t) fb[t] = *reinterpret_cast<const f16x8*>(SB + t * 16 * RB + (ks ? fo1 : fo0));
            }
            const int ad0 = alane ^ (ks << 6), ad1 = alane1 ^ (ks << 6);
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                // 16-row tile (wr, rh, t): image row ir, first pixel x0 (compile-time per (rh, t) and wr)
                const int m16 = (rh * 4 + t) * 16;      // within the wave's row group
                const int ir = wr * (TMW * 16 / W) + m16 / W, x0 = m16 % W;
                const int slot = (int)((unsigned)(sbase + ir) % (unsigned)NS);
                fa[t] = *reinterpret_cast<const f16x8*>(smem + slot * SBYTES + ((G::PAR && (slot & 1)) ? ad1 : ad0) + x0 * RB);
            }
            if (NB == 3 && qq == 0 && !C2D_ABL(p.abl, 1)) sched_piece(cr, ky, 3 * wave + kx, more);   // before the weights
            if (bdeal && !C2D_ABL(p.abl, 1)) {   // (timing ablation 1: no DMA after the prologue)
                if (NB == 3) {
                    constexpr int H0 = (NBP + 1) / 2;
                    if (qq == 0) {
#pragma unroll
                        for (int i = 0; i < H0; ++i) b_piece(ncr, ntap, bw, i);
                    } else {
#pragma unroll
                        for (int i = H0; i < NBP; ++i) b_piece(ncr, ntap, bw, i);
                    }
                } else if (PH == 2) {
                    if (qq == 0) {
#pragma unroll
                        for (int i = 0; i < NBP; ++i) b_piece(ncr, ntap, bw, i);
                    }
                } else {
                    if (qq == 0) { b_piece(ncr, ntap, bw, 0); if (NBP > 1) b_piece(ncr, ntap, bw, 1); }
                    if (qq == 1) { if (NBP > 2) b_piece(ncr, ntap, bw, 2); if (NBP > 3) b_piece(ncr, ntap, bw, 3); }
                    if (qq == 2) { if (NBP > 4) b_piece(ncr, ntap, bw, 4); }
                }
            }
            if (NB == 2 && qq == (PH == 4 ? 2 : 0) && !C2D_ABL(p.abl, 1)) sched_piece(cr, ky, 3 * wave + kx, more);
            if (qq == PH - 1 && nxt) {   // own pieces the next step reads landed
                if (NB == 3 && bdeal) {   // (all but this step's weight pieces)
                    if (NPB % NW == 0 || nbp == NBP) wait_vm_c<NBP>();
                    else wait_vm_c<(NBP > 0 ? NBP - 1 : 0)>();
                } else {
                    wait_vm_c<0>();
                }
            }
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
        bs = NB == 2 ? (bs ^ 1) : (bs == 2 ? 0 : bs + 1);
    }
    if (!sg) C2D_BAR();   // balance the stagger
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
            const int m = mw0 + b * 16 + l15;
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                const int j = nw0 + a * 16 + 4 * lg;
                if (m < p.M && j < p.cout) store_partial(p, slice, m, j, acc[a][b]);
            }
        }
        return;
    }
    // LDS-staged epilogue, as igemm_pp16.h
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
                    *reinterpret_cast<f32x4*>(img + (bb * 16 + l15) * PITCHF + a * 16 + 4 * lg) = acc[a][b0 + bb];
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
            epi_rows_plain<32, TN * 16>(p, img, PITCHF, mw0 + b0 * 16, nw0, lane);
            __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
            __builtin_amdgcn_wave_barrier();
        }
    } else if (p.gn_mom) {   // + the output's GroupNorm moments (c2d_conv_desc::gn_mom)
        constexpr int PITCHB = BN + 4;
        float* img = reinterpret_cast<float*>(smem);
        const int wr0 = wr * 32, wc0 = wc * TN * 16;
        epi_gn_moments<TMW / 2, NRG * 32, BN, BM, TMW * 16>(p, img, PITCHB, m0, n0, tid, [&](auto pass) __attribute__((always_inline)) {
            constexpr int b0 = 2 * decltype(pass)::value;
            f32x4 bv[TN];
#pragma unroll
            for (int a = 0; a < TN; ++a) bv[a] = bias4(p, nw0 + a * 16 + 4 * lg);
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                for (int a = 0; a < TN; ++a)
                    *reinterpret_cast<f32x4*>(img + (wr0 + bb * 16 + l15) * PITCHB + wc0 + a * 16 + 4 * lg) =
                        acc[a][b0 + bb] + bv[a];
        });
    } else {
        constexpr int PITCHB = BN + 4;
        float* img = reinterpret_cast<float*>(smem);
        const int wr0 = wr * 32, wc0 = wc * TN * 16;
        static_for<0, TMW / 2>([&](auto pass) __attribute__((always_inline)) {
            constexpr int b0 = 2 * decltype(pass)::value;
            epi_pass<NRG * 32, BN, true, 512, TMW * 16>(p, img, PITCHB, m0 + b0 * 16, n0, tid, [&]() __attribute__((always_inline)) {
                f32x4 bv[TN];
#pragma unroll
                for (int a = 0; a < TN; ++a) bv[a] = bias4(p, nw0 + a * 16 + 4 * lg);
#pragma unroll
                for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                    for (int a = 0; a < TN; ++a)
                        *reinterpret_cast<f32x4*>(img + (wr0 + bb * 16 + l15) * PITCHB + wc0 + a * 16 + 4 * lg) =
                            acc[a][b0 + bb] + bv[a];
            });
        });
    }
}

// LDS of a row-ring tile: the row slots + the weight ring, or the epilogue images
template <int TN, int W, int TMW, int NB, int NRG>
constexpr int pp16r_smem() {
    constexpr int BN = (8 / NRG) * TN * 16;
    constexpr int ring = RrGeo<W, NRG * TMW * 16>::A_BYTES + NB * BN * 128;
    constexpr int epi_wg = NRG * 32 * (BN + 4) * 4, epi_wv = 8 * 32 * (TN * 16 + 4) * 4;
    constexpr int epi = epi_wg > epi_wv ? epi_wg : epi_wv;
    return ring > epi ? ring : epi;
}

// (output width, 16-row tiles per wave, row groups) of row-ring tile `id`
struct RrTile { int id, w, tmw, nrg; };
constexpr RrTile kRrTiles[] = {{42, 64, 8, 2}, {43, 32, 4, 2}, {44, 16, 4, 2}};

// A row-ring tile applies to: 3x3, stride 1, a single zero-bordered source (src_pad: the host
// maps it to a valid conv, pad 0, over the padded image), 64-channel blocks, output width W
// (64 / 32 / 16), whole BM-row tiles of one image, split-K by whole channel blocks.
// Returns the tile id for this output width, 0 if none.
__host__ __device__ constexpr int pp16r_tile_for(int ksize, int stride, int pad, int c1, int cin, int ow, int oh,
                                                 int w) {
    if (!(ksize == 3 && stride == 1 && pad == 0 && c1 == 0 && cin % 64 == 0 && w == ow + 2)) return 0;
    for (const RrTile& t : kRrTiles)
        if (ow == t.w && (oh * ow) % (t.nrg * t.tmw * 16) == 0) return t.id;   // the first (preferred) tile
    return 0;
}

template <int TN, int W, int TMW, int PH, int NB, int NRG = 2>
static void run_pp16r_t(IgemmParams& p, hipStream_t s) {
    constexpr int BN = (8 / NRG) * TN * 16, BM = NRG * TMW * 16;
    constexpr int smem = pp16r_smem<TN, W, TMW, NB, NRG>();
    static_assert(smem <= 160 * 1024, "LDS ring / epilogue image too large");
    p.gx = (p.cout + BN - 1) / BN;
    p.gy = p.M / BM;
    // K steps per slice: whole channel blocks (9 steps each)
    const int ncb = p.cin / 64;
    int cbs = (p.nkt + 8) / 9;
    if (cbs < 1) cbs = 1;
    if (cbs > ncb) cbs = ncb;
    p.ksplit = (ncb + cbs - 1) / cbs;
    p.nkt = 9 * cbs;
    ensure_lds<igemm_pp16r_kernel<TN, PH, W, TMW, NB, NRG>>(smem);
    hipLaunchKernelGGL((igemm_pp16r_kernel<TN, PH, W, TMW, NB, NRG>), dim3(p.gx * p.gy * p.ksplit), dim3(512), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

#ifndef C2D_PP16R_PH
#define C2D_PP16R_PH 4
#endif
#ifndef C2D_PP16R_NB43
#define C2D_PP16R_NB43 3   // tile 43's weight ring depth (2: the plain 2-phase form, A/B builds)
#endif
#ifndef C2D_PP16R_NB44
#define C2D_PP16R_NB44 3
#endif

template <int TN>
static void run_pp16r(IgemmParams& p, int id, hipStream_t s) {
    if (id == 43) run_pp16r_t<TN, 32, 4, 2, C2D_PP16R_NB43>(p, s);
    else if (id == 44) run_pp16r_t<TN, 16, 4, 2, C2D_PP16R_NB44>(p, s);
    else run_pp16r_t<TN, 64, 8, C2D_PP16R_PH, 2>(p, s);
}

}  // namespace c2d
