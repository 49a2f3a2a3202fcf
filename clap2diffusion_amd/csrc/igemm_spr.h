// Row-ring software-pipelined 3x3 conv (tile 62; included by igemm.hip after igemm_sp.h; uses
// IgemmParams, rr_swz / pp16r_shape_ok (igemm_pp16r.h), sp_epilogue, wait_vm_c, make_rsrc,
// dma_piece, kOOB, C2D_STAMP).
//
// Why: the software-pipelined tile 60 (igemm_sp.h) spends ~4600 cycles per K step against
// ~2560 of MFMA work.  Its timeline stamps with parts of the DMA removed (scripts/sp_stamps.py:
// no DMA 3460, no A pieces 3660, no B pieces 4520 cycles per step) put the excess on the im2col A
// pieces -- 32 KiB per step gathered from the activation, ~26 % of it missing L2 -- not on the
// 40 KiB of L2-resident weights: an A piece holds its loader wave's issue ~450 cycles.
// What: tile 60's wave grid, MFMA groups, fragment-read schedule and two barriers per step, with
// tile 42's A staging (igemm_pp16r.h): on the zero-bordered source [n][h + 2][w + 2][c] a 256-row
// tile at w = 64 is 4 image rows, whose 9 taps per 64-channel block read 6 padded rows, staged
// ONCE per channel block into 8 LDS row slots (slot (c, j) = (6 c + j) & 7, rows 4, 5 of block c
// during its ky = 0 steps, rows 0, 2 / 1, 3 of block c + 1 during its ky = 1 / 2 steps), each
// tap's A fragment a row-shifted read: 6 A pieces per K step instead of 32.
// Loads: four loader waves (0-3) deal each K step's batch -- its 40 weight pieces and the A row
// pieces tile 42 loads one step earlier -- in groups 14-15 of the step two before it and 0-3 of
// the step before (two pieces per group), waited (vmcnt(0)) before X1 of the step before.
// RAW: a row loaded with batch s + 1 is first read by a step >= s + 1 (tile 42's rows load one ky
// phase ahead), whose fragments are read after X1 of step s.  WAR: batch s + 1 goes out after X2 of
// step s - 1 (every read of step <= s - 1 complete), and its rows overwrite slots last read in an
// earlier ky phase than step s's, i.e. by steps <= s - 1; its weights overwrite the weight slot of
// step s - 1.
#pragma once

namespace c2d {

template <int TN>
__global__ void __launch_bounds__(512) igemm_spr_kernel(IgemmParams p) {
    constexpr int BK = 64, TMW = 8, BM = 256, BN = 4 * TN * 16, RB = 2 * BK;
    constexpr int NSLOT = 8, SROWS = 80, SBYTES = SROWS * RB;   // A row slots (72 rows loaded)
    constexpr int A_BYTES = NSLOT * SBYTES;                     // 81,920
    constexpr int BSTAGE = BN * RB;                             // one weight slot
    constexpr int NBL = BN / 32;                                // weight pieces per loader wave per step
    static_assert(A_BYTES + 2 * BSTAGE <= 160 * 1024, "row slots + weight ring");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wave >> 2, wc = wave & 3;
    const int l15 = lane & 15, lg = lane >> 4, lrow = lane >> 3, lchunk = lane & 7;
    const int bid = xcd_remap(blockIdx.x, p.gx * p.gy * p.ksplit);
    const int tile = bid / p.ksplit, slice = bid - tile * p.ksplit;
    const int mt = tile / p.gx, nt = tile - mt * p.gx;
    const int m0 = mt * BM, n0 = nt * BN;
    const int cin = p.cin;
    const int ncb_all = cin / BK, cbs = p.nkt / 9;
    const int cb0 = slice * cbs, ncb = min(ncb_all, cb0 + cbs) - cb0;
    const int nsteps = 9 * (ncb > 0 ? ncb : 0);
    // output tile = 4 whole image rows of image nimg from row y0 (host: ow = 64, oh * ow % 256 == 0)
    const int hw = p.oh * p.ow;
    const int nimg = m0 / hw, y0 = (m0 - nimg * hw) / p.ow;
    const int prow0 = (nimg * p.h + y0) * p.w;   // padded pixel of relative row 0 (p.h, p.w padded)
    const unsigned a_img = 2u * (unsigned)(prow0 * cin + cb0 * BK), a_rowb = 2u * (unsigned)(p.w * cin);
    const char* u_src = uniform_ptr(p.src0);
    const char* u_wt = uniform_ptr(p.wt);
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(u_src, (unsigned)((size_t)p.n * p.h * p.w * cin * 2));
    const unsigned wbytes = (unsigned)((size_t)p.cout * p.kpad * 2);
    // A piece lane offsets (tile 42): pixel lrow of the piece, chunk lchunk ^ rr_swz(row), the two
    // parities of the piece index
    const unsigned a_lo0 = (unsigned)(2 * (lrow * cin + ((lchunk ^ rr_swz(lrow)) << 3)));
    const unsigned a_lo1 = (unsigned)(2 * (lrow * cin + ((lchunk ^ rr_swz(8 + lrow)) << 3)));
    // weight pieces of loader wave d = wave & 3: LDS slots d + 4 k, rows 32 apart
    const int dw = wave & 3;
    const bool loader = wave < 4;
    const int bch = (lchunk ^ ((4 * dw + (lrow >> 1)) & 7)) * 8;
    const int b_row0 = n0 + dw * 8 + lrow;
    const unsigned b_off0 = (unsigned)(b_row0 * 2 * p.kpad + 2 * bch);
    // B fragment offsets (16x16x32: 16 rows x 8 k per lane group, k32 halves)
    const int fo0 = lds_sw<BK>(l15, lg), fo1 = lds_sw<BK>(l15, 4 + lg);
    const int b_off0f = A_BYTES + wc * TN * 16 * RB + fo0, b_off1f = A_BYTES + wc * TN * 16 * RB + fo1;

    // K step s (relative, 0..nsteps-1) = (channel block cr, tap): weight slot s & 1
    auto b_piece = [&](int s, int k) __attribute__((always_inline)) {   // weight piece k of step s
        const int cr = s / 9, tap = s - cr * 9;
        const int k0 = tap * cin + (cb0 + cr) * BK;
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(u_wt + 2 * k0, wbytes - 2 * k0);
        const bool ok = b_row0 + 32 * k < p.cout;
        dma_piece(rb, smem + A_BYTES + (s & 1) * BSTAGE + (dw + 4 * k) * 1024,
                  ok ? b_off0 + (unsigned)(k * 64 * p.kpad) : kOOB);
    };
    // A row piece q (0..5) of the rows tile 42 loads during step s: ky phase rows of block cr / cr + 1
    auto a_count = [&](int s) __attribute__((always_inline)) {   // 6 or 0 pieces
        const int cr = s / 9, ky = (s - cr * 9) / 3;
        return (ky == 0 || cr + 1 < ncb) ? 6 : 0;
    };
    auto a_piece = [&](int s, int q) __attribute__((always_inline)) {
        const int cr = s / 9, tap = s - cr * 9, ky = tap / 3, kx = tap - ky * 3;
        const int qq = 6 * kx + q, arow = qq >= 9 ? 1 : 0, k = qq - 9 * arow;
        const int acr = ky == 0 ? cr : cr + 1;
        const int aj = ky == 0 ? 4 + arow : (ky == 1 ? 2 * arow : 1 + 2 * arow);
        const int slot = (6 * acr + aj) & 7;
        const unsigned soff = a_img + (unsigned)aj * a_rowb + 2u * (unsigned)(8 * k * cin + acr * BK);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lptr_t)(smem + slot * SBYTES + k * 1024), 16, (k & 1) ? a_lo1 : a_lo0,
                                                 (int)soff, 0, 0);
    };
    // batch u = the weights of step u + the A rows loaded "during step u - 1"; loader wave d's
    // pieces: its A pieces first (q = d, d + 4 of the 6), then its NBL weight pieces
    auto batch_n = [&](int u) __attribute__((always_inline)) {
        const int na = u >= 1 ? a_count(u - 1) : 0;
        return (na > dw ? 1 : 0) + (na > dw + 4 ? 1 : 0) + NBL;
    };
    auto batch_piece = [&](int u, int i) __attribute__((always_inline)) {   // wave-uniform
        const int na = u >= 1 ? a_count(u - 1) : 0;
        const int mine = (na > dw ? 1 : 0) + (na > dw + 4 ? 1 : 0);
        if (i < mine) a_piece(u - 1, dw + 4 * i);
        else if (i - mine < NBL) b_piece(u, i - mine);
    };

    f32x4 acc[TN][TMW];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TMW; ++b) acc[a][b] = (f32x4){0.f, 0.f, 0.f, 0.f};

#define C2D_BAR() do { asm volatile("" ::: "memory"); __builtin_amdgcn_s_barrier(); asm volatile("" ::: "memory"); } while (0)
#define C2D_LGKM(N) __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | ((N) << 8) | (3 << 14))
    C2D_STAMP(0);
    // prologue: rows 0..3 of the first block (36 pieces, 9 per loader wave), batch 0 (weights of
    // step 0), then pieces 0-3 of batch 1; wait for all but those 4
    if (loader && nsteps > 0) {
        for (int q = dw; q < 36; q += 4) {
            const int j = q / 9, k = q - 9 * j;
            const unsigned soff = a_img + (unsigned)j * a_rowb + 2u * (unsigned)(8 * k * cin);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lptr_t)(smem + j * SBYTES + k * 1024), 16,
                                                     (k & 1) ? a_lo1 : a_lo0, (int)soff, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < NBL; ++k) b_piece(0, k);
        if (nsteps > 1) {
            const int n1 = batch_n(1);
            for (int i = 0; i < 4 && i < n1; ++i) batch_piece(1, i);
            if (n1 >= 4) wait_vm_c<4>();
            else wait_vm_c<0>();
        } else {
            wait_vm_c<0>();
        }
    }
    C2D_BAR();
    C2D_STAMP(1);

    // A fragment address of row tile b (image row 2 wr + (b >> 2), pixels 16 (b & 3) ..) at tap (ky, kx)
    // of block cr and k32 half ks: slot of padded row 2 wr + (b >> 2) + ky, LDS row 16 (b & 3) + l15 + kx
    struct AAddr { int base0, base1, ck0, ck1; };
    auto a_addr = [&](int s) __attribute__((always_inline)) {
        const int cr = s / 9, tap = s - cr * 9, ky = tap / 3, kx = tap - ky * 3;
        const int ar = l15 + kx, asw = rr_swz(ar & 15);
        AAddr r;
        r.base0 = ((6 * cr + 2 * wr + ky) & 7) * SBYTES + ar * RB;
        r.base1 = ((6 * cr + 2 * wr + 1 + ky) & 7) * SBYTES + ar * RB;
        r.ck0 = (lg ^ asw) << 4;
        r.ck1 = ((lg + 4) ^ asw) << 4;
        return r;
    };
    auto a_read = [&](const AAddr& r, int g3) __attribute__((always_inline)) {   // g3 constant after unrolling
        const int ks3 = g3 >> 3, b3 = g3 & 7;
        return *reinterpret_cast<const f16x8*>(smem + ((b3 >> 2) ? r.base1 : r.base0) + (ks3 ? r.ck1 : r.ck0) +
                                               (b3 & 3) * 16 * RB);
    };

    f16x8 fb0[TN], fb1[TN], fa[4];
    {
        const AAddr r0 = a_addr(0);
#pragma unroll
        for (int t = 0; t < TN; ++t) fb0[t] = *reinterpret_cast<const f16x8*>(smem + b_off0f + t * 16 * RB);
#pragma unroll
        for (int t = 0; t < 3; ++t) fa[t] = a_read(r0, t);
    }

    for (int s = 0; s < nsteps; ++s) {
        const int bs = s & 1;
        const char* SB = smem + bs * BSTAGE;                // this step's weight slot (+ A_BYTES in offsets)
        const char* SBn = smem + (bs ^ 1) * BSTAGE;         // the next step's (read after X1)
        const bool nxt = s + 1 < nsteps, nxt2 = s + 2 < nsteps;
        const AAddr rc = a_addr(s), rn = a_addr(s + 1);     // rn only read after X1, and only if nxt
        const int n1 = nxt ? batch_n(s + 1) : 0, n2 = nxt2 ? batch_n(s + 2) : 0;
        C2D_LGKM(0);
        C2D_STAMP(4 + 6 * s);
        static_for<0, 16>([&](auto G) __attribute__((always_inline)) {
            constexpr int g = decltype(G)::value;
            constexpr int ks = g >> 3, b = g & 7;
            // ---- LDS reads ahead of use (tile 60's schedule; the next step's after X1)
            if constexpr (g + 3 < 16) fa[(g + 3) & 3] = a_read(rc, g + 3);
            else fa[(g + 3 - 16) & 3] = a_read(rn, g + 3 - 16);
            if constexpr (g >= 1 && g <= TN) fb1[g - 1] = *reinterpret_cast<const f16x8*>(SB + b_off1f + (g - 1) * 16 * RB);
            if constexpr (g >= 11 && g <= 14) {
                constexpr int t0 = g == 11 ? 0 : g - 10, t1 = g == 11 ? 2 : g - 9;
#pragma unroll
                for (int t = t0; t < t1 && t < TN; ++t) fb0[t] = *reinterpret_cast<const f16x8*>(SBn + b_off0f + t * 16 * RB);
            }
            // ---- MFMAs (loader waves deal two batch pieces after the first)
            const f16x8 av = fa[g & 3];
#pragma unroll
            for (int a = 0; a < TN; ++a) {
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ks ? fb1[a] : fb0[a], av, acc[a][b], 0, 0, 0);
                if (a == 0 && loader && !(C2D_SP_ABL & 1)) {
                    if constexpr (g < 8) {   // batch s + 1: pieces 4 + 2 g, 5 + 2 g
                        if (4 + 2 * g < n1) batch_piece(s + 1, 4 + 2 * g);
                        if (5 + 2 * g < n1) batch_piece(s + 1, 5 + 2 * g);
                    }
                    if constexpr (g >= 14) {   // batch s + 2: pieces 0-3, after X2
                        if (2 * (g - 14) < n2) batch_piece(s + 2, 2 * (g - 14));
                        if (2 * (g - 14) + 1 < n2) batch_piece(s + 2, 2 * (g - 14) + 1);
                    }
                }
            }
            if constexpr (g == 10) {   // X1: batch s + 1 landed (weights of step s + 1, rows it reads)
                C2D_STAMP(5 + 6 * s);
                wait_vm_c<0>();
                C2D_BAR();
                C2D_STAMP(6 + 6 * s);
            }
            if constexpr (g == 13) {   // X2: every read of step s done (A(15): group 12; >= 2 reads after it)
                C2D_LGKM(2);
                C2D_BAR();
                C2D_STAMP(7 + 6 * s);
            }
            if constexpr (g == 14) C2D_STAMP(8 + 6 * s);
            if constexpr (g == 15) C2D_STAMP(9 + 6 * s);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
#undef C2D_BAR
#undef C2D_LGKM
    C2D_STAMP(2);
    sp_epilogue<TN>(p, acc, m0, n0, slice, wave, lane, tid, smem);
    C2D_STAMP(3);
}

template <int TN>
static void run_spr(IgemmParams& p, hipStream_t s) {
    constexpr int BN = 4 * TN * 16;
    constexpr int ring = 8 * 80 * 128 + 2 * BN * 128;
    constexpr int epi_wg = 64 * (BN + 4) * 4, epi_wv = 8 * 32 * (TN * 16 + 4) * 4;
    constexpr int epi = epi_wg > epi_wv ? epi_wg : epi_wv;
    constexpr int smem = ring > epi ? ring : epi;
    static_assert(smem <= 160 * 1024, "LDS row slots / epilogue image too large");
    p.gx = (p.cout + BN - 1) / BN;
    p.gy = p.M / 256;
    // K steps per slice: whole channel blocks (9 steps each)
    const int ncb = p.cin / 64;
    int cbs = (p.nkt + 8) / 9;
    if (cbs < 1) cbs = 1;
    if (cbs > ncb) cbs = ncb;
    p.ksplit = (ncb + cbs - 1) / cbs;
    p.nkt = 9 * cbs;
    ensure_lds<igemm_spr_kernel<TN>>(smem);
    hipLaunchKernelGGL((igemm_spr_kernel<TN>), dim3(p.gx * p.gy * p.ksplit), dim3(512), smem, s, p);
    if (p.ksplit > 1) run_splitk_reduce(p, s);
}

}  // namespace c2d
