// Row-ring ping-pong 3x3 conv (tile 42; included by igemm.hip after igemm_pps.h; uses
// IgemmParams, lds_sw, wait_vm_c, make_rsrc, kOOB, store_partial, epi_pass, epi_rows_plain).
//
// Why: the one-shot ping-pong conv (igemm_pp16.h, tile 40) stages, per 64-deep K step, a
// 256-row A tile (one 3x3 tap of one 64-channel block) and a 320-row weight tile: 72 LDS-DMA
// pieces of 1 KiB, 9 per wave, each holding its wave's issue for 60-185 cycles -- the load
// section of every phase is as long as the partner's MFMA section (MFMA busy 0.48).  The nine
// taps of one channel block re-read, from L2, nine shifted copies of the same few image rows.
//
// What: the input is the zero-bordered layout [n][h + 2][w + 2][c] (c2d_conv_desc::src_pad,
// written by c2d_groupnorm_pad), so every tap of every output pixel is in bounds: the conv is a
// "valid" 3x3 over the padded image and needs no masks.  A 256-row output tile at w = 64 is
// R = 4 whole image rows; the 9 K steps of a channel block read R + 2 = 6 padded image rows,
// staged ONCE per channel block into a ring of 2R = 8 row slots (80 LDS rows of 128 B: 66
// padded pixels x 64 channels, 72 loaded), and every tap's A fragment is a row-shifted read of them:
// 6 A pieces per K step instead of 32 (46 DMA pieces per K step instead of 72).
//   Row schedule (rows of channel block c, relative j = 0..5 = padded rows y0 .. y0 + 5;
//   slot (c, j) = (6c + j) mod 8), two rows per 3-step ky phase:
//     ky = 0 of c: (c, 4), (c, 5)            ky = 1: (c+1, 0), (c+1, 2)      ky = 2: (c+1, 1), (c+1, 3)
//   each into the slot of a row whose last tap ran in an earlier ky phase (row j is read by
//   the taps ky in [j - 3, j]), and each landed (vmcnt(0) + barrier) before its first tap.
//   The prologue stages rows (0, 0..3).
// LDS: 8 row slots of 80 rows (81,920 B; 72 rows loaded) + a 2-slot weight ring (2 x 40 KiB) =
// 160 KiB, all of it.  The A slots use their own bank swizzle (rr_swz), conflict-free for the
// three kx row shifts, repeating every 16 rows: a tap's fragment address is one per-lane base per
// (kx, k32 half) plus ds_read immediates for the 16-row tiles.
// The MFMA / phase / barrier structure is igemm_pp16.h's (4 phases per K step: (k32 half,
// row half); the two row groups one barrier apart; next-step pieces dealt in phases 0-2,
// waited in phase 3); a row half of a wave's 128 rows is one image row, so each phase's A
// fragments come from one row slot.  Split-K slices own whole channel blocks.
#pragma once

namespace c2d {

// Bank swizzle of the A row slots: 16-B chunk c of LDS row r sits at slot c ^ rr_swz(r mod 16).
// The fragment reads of a tap start at row kx in {0, 1, 2} of each 16-row group; the standard
// (r >> 1) & 7 swizzle is conflict-free only for kx = 0 (2-way at kx = 1, 2: 8 LDS cycles per
// ds_read_b128 instead of 4).  This table (found by exhaustive search over the ds_read_b128
// lane groups, MI355X_MICROARCH.md §LDS) is conflict-free for all three shifts and both k32
// halves; it repeats every 16 rows, so slots are 80 rows apart (a multiple of 16) and the
// 16-row tiles stay ds_read immediates.
__device__ __forceinline__ int rr_swz(int r) {
    // f = {0,0,1,1,2,2,4,4, 5,5,6,6,2,2,6,6}, 3 bits per row
    constexpr unsigned long long F = 0ull | (0ull << 3) | (1ull << 6) | (1ull << 9) | (2ull << 12) | (2ull << 15) |
                                     (4ull << 18) | (4ull << 21) | (5ull << 24) | (5ull << 27) | (6ull << 30) |
                                     (6ull << 33) | (2ull << 36) | (2ull << 39) | (6ull << 42) | (6ull << 45);
    return (int)((F >> (3 * r)) & 7ull);
}

#ifndef C2D_PP16R_PH
#define C2D_PP16R_PH 4
#endif

// PH phases per K step: 4 = (k32 half, row half), 20-MFMA sections; 2 = k32 half, 40-MFMA
// sections with every DMA piece of the step dealt in phase 0 (phase 1 is their landing time)
template <int TN, int PH>
__global__ void __launch_bounds__(512) igemm_pp16r_kernel(IgemmParams p) {
    static_assert(PH == 2 || PH == 4, "pp16r phases per K step");
    constexpr int BK = 64, TMW = 8, RT = PH == 4 ? 4 : 8, NW = 8;
    constexpr int BM = 256, BN = 4 * TN * 16;
    constexpr int RB = 2 * BK;                    // bytes per LDS row
    constexpr int NSLOT = 8, SROWS = 80, SBYTES = SROWS * RB;   // 72 rows used; stride a multiple of 16
    constexpr int A_BYTES = NSLOT * SBYTES;       // 81,920
    constexpr int BSTAGE = BN * RB;
    constexpr int NBP = BN / 8 / NW;              // weight pieces per wave per K step
    static_assert(NBP * 8 * NW == BN, "weight rows must split evenly over the waves");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int l15 = lane & 15, lg = lane >> 4;
    const int lrow = lane >> 3, lchunk = lane & 7;
    const int bid = xcd_remap(blockIdx.x, p.gx * p.gy * p.ksplit);
    const int tile = bid / p.ksplit, slice = bid - tile * p.ksplit;
    const int mt = tile / p.gx, nt = tile - mt * p.gx;
    const int m0 = mt * BM, n0 = nt * BN;
    const int cin = p.cin;
    const int ncb_all = cin / BK, cbs = p.nkt / 9;
    const int cb0 = slice * cbs, ncb = min(ncb_all, cb0 + cbs) - cb0;
    // output tile = 4 whole image rows of image nimg starting at row y0 (host: ow = 64, oh * ow % 256 == 0)
    const int hw = p.oh * p.ow;
    const int nimg = m0 / hw, y0 = (m0 - nimg * hw) / p.ow;
    const int prow0 = (nimg * p.h + y0) * p.w;    // padded pixel index of relative row j = 0
    const unsigned a_img = 2u * (unsigned)(prow0 * cin + cb0 * BK), a_rowb = 2u * (unsigned)(p.w * cin);

    const char* u_src = uniform_ptr(p.src0);
    const char* u_wt = uniform_ptr(p.wt);
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(u_src, (unsigned)((size_t)p.n * p.h * p.w * cin * 2));
    const unsigned wbytes = (unsigned)((size_t)p.cout * p.kpad * 2);

    // A piece lane offsets: pixel lrow of the piece, logical chunk lchunk ^ rr_swz(row) so the
    // lane-linear image is swizzled (rows 8k + lrow: the parity of piece k picks the half)
    const unsigned a_lo0 = (unsigned)(2 * (lrow * cin + ((lchunk ^ rr_swz(lrow)) << 3)));
    const unsigned a_lo1 = (unsigned)(2 * (lrow * cin + ((lchunk ^ rr_swz(8 + lrow)) << 3)));
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
        const int s = (6 * cr + j) & 7;
        const unsigned soff = a_img + (unsigned)j * a_rowb + 2u * (unsigned)(8 * k * cin + cr * BK);
        const unsigned lo = (k & 1) ? a_lo1 : a_lo0;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lptr_t)(smem + s * SBYTES + k * 1024), 16, lo, (int)soff, 0, 0);
    };
    // weight piece i of K step (cr, tap) into ring slot bs
    auto b_piece = [&](int cr, int tap, int bs, int i) __attribute__((always_inline)) {
        const int k0 = tap * cin + (cb0 + cr) * BK;
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(u_wt + 2 * k0, wbytes - 2 * k0);
        dma_piece(rb, smem + A_BYTES + bs * BSTAGE + (wave + i * NW) * 1024, b_off[i]);
    };

    f32x4 acc[TN][TMW];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TMW; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

#define C2D_BAR() do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
    // prologue: rows 0..3 of the first channel block (36 pieces) and the weights of step 0
    if (ncb > 0) {
        for (int q = wave; q < 36; q += NW) a_piece(0, q / 9, q - (q / 9) * 9);
#pragma unroll
        for (int i = 0; i < NBP; ++i) b_piece(0, 0, 0, i);
    }
    wait_vm_c<0>();
    C2D_BAR();
    if (wr) C2D_BAR();   // group 1 runs one barrier behind group 0

    f16x8 fa[RT], fb[TN];
    const int nsteps = 9 * ncb;
    for (int kt = 0; kt < nsteps; ++kt) {
        const int cr = kt / 9, tap = kt - cr * 9, ky = tap / 3, kx = tap - ky * 3;
        const bool more = cr + 1 < ncb;
        const int bs = kt & 1;                          // weight ring slot of this step
        const bool nxt = kt + 1 < nsteps;
        const int ncr = tap < 8 ? cr : cr + 1, ntap = tap < 8 ? tap + 1 : 0;
        // this step's A piece (waves 0..5): piece 6 kx + wave of the ky phase's two rows
        const int q = 6 * kx + wave;
        const bool a_on = wave < 6 && (ky == 0 || more);
        const int arow = q < 9 ? 0 : 1, ak = q - arow * 9;
        const int a_cr = ky == 0 ? cr : cr + 1;
        const int a_j = ky == 0 ? 4 + arow : (ky == 1 ? 2 * arow : 1 + 2 * arow);
        const char* SB = smem + A_BYTES + bs * BSTAGE + wc * TN * 16 * RB;
        // A fragment rows: row l15 + kx of each 16-row group of the row slot of row half rh
        // (image row 2 wr + rh + ky of channel block cr)
        const int ar = l15 + kx, asw = rr_swz(ar & 15);
        int asb[2];
#pragma unroll
        for (int rh = 0; rh < 2; ++rh) asb[rh] = ((6 * cr + 2 * wr + rh + ky) & 7) * SBYTES + ar * RB;
#pragma unroll
        for (int qq = 0; qq < PH; ++qq) {
            const int ks = PH == 4 ? qq >> 1 : qq, rh = PH == 4 ? qq & 1 : 0;
            // ---- load section
            if (rh == 0) {
#pragma unroll
                for (int t = 0; t < TN; ++t) fb[t] = *reinterpret_cast<const f16x8*>(SB + t * 16 * RB + (ks ? fo1 : fo0));
            }
#pragma unroll
            for (int hh = 0; hh < RT / 4; ++hh) {   // the row halves of this phase (one image row each)
                const int ad = asb[rh + hh] + (((lg + 4 * ks) ^ asw) << 4);
#pragma unroll
                for (int t = 0; t < 4; ++t) fa[hh * 4 + t] = *reinterpret_cast<const f16x8*>(smem + ad + t * 16 * RB);
            }
            if (nxt && !C2D_ABL(p.abl, 1)) {   // (timing ablation 1: no DMA after the prologue)
                if (PH == 2) {
                    if (qq == 0) {
#pragma unroll
                        for (int i = 0; i < NBP; ++i) b_piece(ncr, ntap, bs ^ 1, i);
                    }
                } else {
                    if (qq == 0) { b_piece(ncr, ntap, bs ^ 1, 0); if (NBP > 1) b_piece(ncr, ntap, bs ^ 1, 1); }
                    if (qq == 1) { if (NBP > 2) b_piece(ncr, ntap, bs ^ 1, 2); if (NBP > 3) b_piece(ncr, ntap, bs ^ 1, 3); }
                    if (qq == 2) { if (NBP > 4) b_piece(ncr, ntap, bs ^ 1, 4); }
                }
            }
            if (qq == (PH == 4 ? 2 : 0) && a_on && !C2D_ABL(p.abl, 1)) a_piece(a_cr, a_j, ak);
            if (qq == PH - 1 && nxt) wait_vm_c<0>();   // own pieces of later steps landed
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
    } else {
        constexpr int PITCHB = BN + 4;
        float* img = reinterpret_cast<float*>(smem);
        const int wr0 = wr * 32, wc0 = wc * TN * 16;
        static_for<0, TMW / 2>([&](auto pass) __attribute__((always_inline)) {
            constexpr int b0 = 2 * decltype(pass)::value;
            epi_pass<64, BN, true, 512, TMW * 16>(p, img, PITCHB, m0 + b0 * 16, n0, tid, [&]() __attribute__((always_inline)) {
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

// LDS of tile 42: the 8 row slots + the 2-slot weight ring, or the epilogue images
template <int TN>
constexpr int pp16r_smem() {
    constexpr int ring = 8 * 80 * 128 + 2 * (4 * TN * 16) * 128;
    constexpr int epi_wg = 64 * (4 * TN * 16 + 4) * 4, epi_wv = 8 * 32 * (TN * 16 + 4) * 4;
    constexpr int epi = epi_wg > epi_wv ? epi_wg : epi_wv;
    return ring > epi ? ring : epi;
}

// Tile 42 applies to: 3x3, stride 1, a single zero-bordered source (src_pad: the host maps it
// to a valid conv, pad 0, over the padded image), 64-channel blocks, output width 64, whole
// 256-row tiles, split-K by whole channel blocks.
__host__ __device__ constexpr bool pp16r_shape_ok(int ksize, int stride, int pad, int c1, int cin, int ow, int oh,
                                                  int w) {
    return ksize == 3 && stride == 1 && pad == 0 && c1 == 0 && cin % 64 == 0 && ow == 64 && w == ow + 2 &&
           (oh * ow) % 256 == 0;
}

template <int TN>
static void run_pp16r(IgemmParams& p, hipStream_t s) {
    constexpr int BN = 4 * TN * 16;
    constexpr int smem = pp16r_smem<TN>();
    static_assert(smem <= 160 * 1024, "LDS ring / epilogue image too large");
    p.gx = (p.cout + BN - 1) / BN;
    p.gy = p.M / 256;
    // K steps per slice: whole channel blocks (9 steps each)
    const int ncb = p.cin / 64;
    int cbs = (p.nkt + 8) / 9;
    if (cbs < 1) cbs = 1;
    if (cbs > ncb) cbs = ncb;
    p.ksplit = (ncb + cbs - 1) / cbs;
    p.nkt = 9 * cbs;
    ensure_lds<igemm_pp16r_kernel<TN, C2D_PP16R_PH>>(smem);
    hipLaunchKernelGGL((igemm_pp16r_kernel<TN, C2D_PP16R_PH>), dim3(p.gx * p.gy * p.ksplit), dim3(512), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

}  // namespace c2d
