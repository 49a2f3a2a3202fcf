// Panel GEMM (tile 70): 1x1 conv / linear with K = 320 or 640, for the transformer-block
// projections whose K loop is too short for a per-K-step LDS ring to pay (the GEGLU, QKV, to_q,
// proj_in / proj_out and to_out GEMMs of levels 0 / 1).
//
// One workgroup = 8 waves = a 128-row panel of A, loaded ONCE into LDS by LDS-DMA (all K: 80 KiB
// at K = 320, 160 KiB at 640; XOR-swizzled lane-linear rows as in the DMA tiles), then one
// barrier.  After it the waves never synchronise again: each walks its own 32-column blocks of
// the output (block j = split * 8 + wave, j += 8 * nsplit) over the whole K, reading its A
// fragments from the shared panel and its B (weight) fragments straight from global memory into
// registers through a PD-deep register ring that runs on across column blocks, so the next
// block's first weights are in flight during this block's epilogue.  With two waves per SIMD and
// no barriers, one wave's epilogue (bias, residual, GEGLU) overlaps its partner's MFMAs.
//
// Traffic per 256 columns of a panel (K = 320): LDS reads 8 waves x 80 KiB = 640 KiB (2.5k cycles
// at 256 B/clk) and weight reads 160 KiB (2.5k cycles at the CU's 64 B/clk vector-memory path),
// both under the 5.1k MFMA cycles per SIMD.  The weights are shared by every panel, so they are
// L2 hits after the first panels of each XCD.
//
// Lane roles per 16x16x32 MFMA (C^T = W A^T, so a lane holds 4 consecutive columns of one row,
// stored directly by panel_epilogue): A fragment = rows 16 b + (lane & 15) of the panel,
// channels 32 ks + 8 (lane >> 4) .. +7; B fragment = weight rows (output columns) 32 j + 16 a +
// (lane & 15), same channels.
#pragma once

namespace c2d {

constexpr int kPanelRows = 128;

// Epilogue kinds (compile-time, so the epilogue is straight-line code): plain, + residual,
// GEGLU (tile 0 = h, tile 1 = g of 16 output features).  panel_eligible admits no time embedding
// and no other activation.
enum PanelEpi { PE_PLAIN = 0, PE_RESID = 1, PE_GEGLU = 2 };

// Residual operands of one 128 x 32 block, loaded PD K steps before its epilogue (with the bias) -- ahead of the
// next block's first weight loads, so waiting for them never waits for those
__device__ __forceinline__ void panel_resid(const IgemmParams& p, f16x4 (&rv)[8][2], int m0, int ncol0, int lane) {
    const int lr = lane & 15, jo = ncol0 + 4 * (lane >> 4);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int m = m0 + b * 16 + lr;
        const f16* r = p.resid + (size_t)(m < p.M ? m : 0) * p.resid_ld + jo;
        rv[b][0] = *reinterpret_cast<const f16x4*>(r);
        rv[b][1] = *reinterpret_cast<const f16x4*>(r + 16);
    }
}

// bias of one block's two column tiles: the accumulators of the block start from it (loaded
// during the previous block), so the epilogue adds no bias

__device__ __forceinline__ void panel_bias(const IgemmParams& p, float4 (&bv)[2], int ncol0, int lane) {
    const int jb = ncol0 + 4 * (lane >> 4);
#pragma unroll
    for (int a = 0; a < 2; ++a)
        bv[a] = p.bias ? *reinterpret_cast<const float4*>(p.bias + jb + 16 * a) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Epilogue of one 128 x 32 block (acc[a][b]: column tile a, row tile b; lane holds row
// m0 + 16 b + (lane & 15), columns 4 (lane >> 4) .. +3 of the tile; bias already in acc):
// residual or GEGLU, fp16 stores of 8 B
template <int EPI>
__device__ __forceinline__ void panel_epilogue(const IgemmParams& p, const f32x4 (&acc)[2][8], const f16x4 (&rv)[8][2],
                                               int m0, int ncol0, int lane) {
    const int lr = lane & 15, lc = 4 * (lane >> 4);
    const int jo = EPI == PE_GEGLU ? (ncol0 >> 1) + lc : ncol0 + lc;   // output column of tile 0
    // stores through a buffer descriptor over the output: a row past M gets an offset past
    // num_records and the buffer unit drops it, so no store sits under a branch (a conditional
    // store would make the block loop's header wait for the stores, see igemm_panel_kernel)
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out, (unsigned)((size_t)p.M * p.out_ld * 2));
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const int m = m0 + b * 16 + lr;
        const unsigned off = m < p.M ? (unsigned)(2 * (m * p.out_ld + jo)) : kOOB;
        if constexpr (EPI == PE_GEGLU) {
            f16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (f16)(acc[0][b][r] * gelu_sig(acc[1][b][r]));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ro, off, 0, 0);
        } else {
#pragma unroll
            for (int a = 0; a < 2; ++a) {
                f16x4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float v = acc[a][b][r];
                    if constexpr (EPI == PE_RESID) v += (float)rv[b][a][r];
                    o[r] = (f16)v;
                }
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ro, off + 32 * a, 0, 0);
            }
        }
    }
}

// LayerNorm in place on a landed panel (C2D_PRO_LNFOLD): row r of the 128 is normalised,
// (x - mean) * rstd rounded to fp16 as the LayerNorm kernel's output is, by the four lanes
// 4 (r % 16) .. +3 of wave r / 16: each holds NKB * 2 of the row's NKB * 8 16-B chunks (the
// swizzled image's slots, any order) in registers through both passes (fixed order), the quarters
// combining by two lane exchanges.  Rows past M were DMA'd as zeros and stay zero.  The caller
// synchronises the workgroup before the panel is read.
template <int NKB>
__device__ __forceinline__ void panel_ln_inplace(char* smem, int wave, int lane, float eps) {
    constexpr int BLK = kPanelRows * 128, NC = NKB * 2;
    constexpr float inv_k = 1.0f / (NKB * 64);
    const int row = wave * 16 + (lane >> 2), qd = lane & 3;
    char* rb = smem + (row >> 3) * 1024 + (row & 7) * 128;
    f16x8 v[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        const int c = qd * NC + i;
        v[i] = *reinterpret_cast<const f16x8*>(rb + (c >> 3) * BLK + (c & 7) * 16);
    }
    float sm = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) sm += (float)v[i][e];
    sm += __shfl_xor(sm, 1);
    sm += __shfl_xor(sm, 2);
    const float mean = sm * inv_k;
    float sq = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float d = (float)v[i][e] - mean;
            sq = fmaf(d, d, sq);
        }
    sq += __shfl_xor(sq, 1);
    sq += __shfl_xor(sq, 2);
    const float rstd = 1.0f / sqrtf(sq * inv_k + eps);
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (f16)(((float)v[i][e] - mean) * rstd);
        const int c = qd * NC + i;
        *reinterpret_cast<f16x8*>(rb + (c >> 3) * BLK + (c & 7) * 16) = o;
    }
}

// LNF (C2D_PRO_LNFOLD): a LayerNorm folded in -- once the panel has landed it is normalised in
// place (panel_ln_inplace); the GEMM then runs on W diag(gamma) with bias b + W beta
template <int NK32, int PD, int EPI, bool LNF = false>
__global__ void __launch_bounds__(512) igemm_panel_kernel(IgemmParams p, int nsplit) {
    static_assert(NK32 % PD == 0 && (PD & 1) && !(NK32 & 1), "the register ring restarts with every column block; line pairs");
    constexpr int BM = kPanelRows, NKB = NK32 / 2, BLK = BM * 128;   // bytes per 64-channel block
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int panel = bid / nsplit, split = bid - panel * nsplit;
    const int m0 = panel * BM;

    // ---- A panel -> LDS: piece = 8 rows of one 64-channel block (1 KiB); rows past M read zeros
    {
        const int lrow = lane >> 3, slot = lane & 7;
        const __amdgpu_buffer_rsrc_t ra = make_rsrc(uniform_ptr(p.src0), (unsigned)((size_t)p.M * p.c0 * 2));
        constexpr int RG = BM / 8, PIECES = RG * NKB;
        for (int pc = wave; pc < PIECES; pc += 8) {
            const int kb = pc / RG, rg = pc - kb * RG;
            const int row = rg * 8 + lrow, m = m0 + row;
            const int ch = kb * 64 + ((slot ^ ((row >> 1) & 7)) << 3);
            const unsigned off = m < p.M ? (unsigned)(2 * (m * p.c0 + ch)) : kOOB;
            dma_piece(ra, smem + kb * BLK + rg * 1024, off);
        }
    }

    const int nblk = p.cout >> 5, stride = 8 * nsplit;
    const int j0 = split * 8 + wave;
    // B pointers of a column block: lane's weight row (output column) and its 8-channel group
#ifdef C2D_PANEL_FULLLINE
    // timing diagnostic only (wrong results): every weight load covers 8 whole 128-B lines
    const int brow = lane >> 3, bk = 8 * (lane & 7);
    auto boff = [&](int s) { return (s & 1) * 8 * p.kpad + (s >> 1) * 64; };
#else
    const int brow = lane & 15, bk = 8 * (lane >> 4);
    auto boff = [&](int s) { return 32 * s; };
#endif
    auto bptr = [&](int j, int a) { return p.wt + (size_t)(32 * j + 16 * a + brow) * p.kpad + bk; };
    const int jfirst = j0 < nblk ? j0 : 0;   // idle waves (j0 >= nblk) still reach the barrier
    const f16* pb0 = bptr(jfirst, 0);
    const f16* pb1 = bptr(jfirst, 1);
    f16x8 bq[PD][2];
#pragma unroll
    for (int s = 0; s < PD - 1; ++s) {   // the ring's first PD - 1 steps, in flight under the panel's DMA
        bq[s][0] = *reinterpret_cast<const f16x8*>(pb0 + boff(s));
        bq[s][1] = *reinterpret_cast<const f16x8*>(pb1 + boff(s));
    }
    float4 bv[2];   // bias of the next column block: its accumulators start from it
    panel_bias(p, bv, 32 * jfirst, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if constexpr (LNF) {
        panel_ln_inplace<NKB>(smem, wave, lane, p.pro_eps);
        __syncthreads();
    }
    if (j0 >= nblk) return;   // wave-uniform; no barrier follows
    if (C2D_TUNE_PANEL_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);   // static priority, waves 4-7 (A/B)

    int fa0[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) fa0[kk] = lds_off(lane & 15, kk * 4 + (lane >> 4));

    // A fragments double-buffered by K step parity; step 0's are the same for every column block
    // (same panel rows, same channels), so they carry over the epilogue into the next block.  One
    // sched_barrier per step keeps the compiler from hoisting all the unrolled steps' LDS reads
    // (it otherwise holds the whole panel's fragments and spills).
    f16x8 fa[2][8];
    auto aread = [&](int ks, f16x8 (&dst)[8]) {
        const char* S = smem + (ks >> 1) * BLK + fa0[ks & 1];
#pragma unroll
        for (int b = 0; b < 8; ++b) dst[b] = *reinterpret_cast<const f16x8*>(S + b * 2048);
    };
    aread(0, fa[0]);
    // one column block; the first is peeled off the loop so that the loop header sees the same
    // outstanding memory operations from both of its predecessors (next block's weights, then
    // this block's stores) and waits only for the weights it uses, never for the stores
    auto block = [&](int j) __attribute__((always_inline)) {
        const int jn = j + stride < nblk ? j + stride : j;   // the last block re-reads itself (no branch)
        const f16* pn0 = bptr(jn, 0);
        const f16* pn1 = bptr(jn, 1);
        f32x4 acc[2][8];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 8; ++b) acc[a][b] = (f32x4){bv[a].x, bv[a].y, bv[a].z, bv[a].w};
        f16x4 rv[8][2];
#pragma unroll
        for (int ks = 0; ks < NK32; ++ks) {
            if (ks == NK32 - PD) {   // epilogue operands and the next block's bias, ahead of its first weights
                panel_bias(p, bv, 32 * jn, lane);
                if constexpr (EPI == PE_RESID) panel_resid(p, rv, m0, 32 * j, lane);
            }
            aread(ks + 1 < NK32 ? ks + 1 : 0, fa[(ks + 1) & 1]);
            const f16x8 fb0 = bq[ks % PD][0], fb1 = bq[ks % PD][1];
            // refill: at every even step, both 32-channel halves of one weight line pair -- steps
            // ks + PD - 1 and ks + PD (slots (ks - 1) % PD and ks % PD, both consumed by now), of
            // this block or, past its end, of the next one -- so the two 64-B reads of each 128-B
            // line go out back to back
            if (!(ks & 1)) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int st = ks + PD - 1 + h, sl = st % PD;
#ifndef C2D_PANEL_NOB
                    const f16* q0 = st < NK32 ? pb0 + boff(st) : pn0 + boff(st - NK32);
                    const f16* q1 = st < NK32 ? pb1 + boff(st) : pn1 + boff(st - NK32);
                    bq[sl][0] = *reinterpret_cast<const f16x8*>(q0);
                    bq[sl][1] = *reinterpret_cast<const f16x8*>(q1);
#else
                    (void)sl;   // timing diagnostic only (wrong results): no weight traffic after the prologue
#endif
                }
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                acc[0][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb0, fa[ks & 1][b], acc[0][b], 0, 0, 0);
                acc[1][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb1, fa[ks & 1][b], acc[1][b], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        panel_epilogue<EPI>(p, acc, rv, m0, 32 * j, lane);
        pb0 = pn0;
        pb1 = pn1;
    };
    block(j0);
    for (int j = j0 + stride; j < nblk; j += stride) block(j);
}

#ifdef C2D_PANEL_STAMP
// Diagnostic build only (build.py --variant pstamp --define C2D_PANEL_STAMP): s_memtime stamps of one
// workgroup's waves into a buffer nothing else reads (c2d_debug_panel_stamps copies it out): start,
// after the panel barrier, then per column block its start, each K step after its wait, the end of
// the K loop and the end of the epilogue.  The production library has no stamp code.
constexpr int kPanelStampPer = 2 + 8 * 16;
static __device__ unsigned long long g_panel_stamps[8 * kPanelStampPer];   // per compile unit: read by part 4 only
#define C2D_PSTAMP(idx)                                                                            \
    do {                                                                                          \
        if (blockIdx.x == 77 && lane == 0 && (idx) < kPanelStampPer)                              \
            g_panel_stamps[wave * kPanelStampPer + (idx)] = __builtin_amdgcn_s_memtime();         \
    } while (0)
#else
#define C2D_PSTAMP(idx) do {} while (0)
#endif

template <int N>
__device__ __forceinline__ void panel_wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// K = 320 form with the weights through LDS: per wave a two-slot ring of its 32 weight rows x 64
// channels (4 KiB, four LDS-DMA pieces of 8 whole 128-B lines each) beside the 80 KiB panel, 144
// KiB in all.  A wave reads only its own ring, so the ring needs no barrier: the wave waits for its
// own pieces with a counted vmcnt (everything issued after them may stay in flight: the next
// step's pieces, and at a block's first step the previous block's stores).  Weight fragments
// loaded into registers straight from global memory touch 16 half lines per instruction, which
// measured 20 % slower over the whole kernel than whole-line loads (profiles/r05_panel_gemm.txt).
// Bias and residual go through buffer loads (a missing bias reads zeros past num_records), so
// their count in the vmcnt stream is a compile-time constant.
// LNF (C2D_PRO_LNFOLD): as igemm_panel_kernel's
template <int EPI, bool LNF = false>
__global__ void __launch_bounds__(512) igemm_panel_dma_kernel(IgemmParams p, int nsplit, int stagger) {
    constexpr int BM = kPanelRows, NKB = 5, BLK = BM * 128, A_BYTES = NKB * BLK, BSLOT = 32 * 128;
    constexpr int NST = EPI == PE_GEGLU ? 8 : 16;          // stores per block
    constexpr int NRES = EPI == PE_RESID ? 18 : 2;         // bias (2) + residual (16) loads per block
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int panel = bid / nsplit, split = bid - panel * nsplit;
    const int m0 = panel * BM;
    const int lrow = lane >> 3, lslot = lane & 7;
    C2D_PSTAMP(0);
    {   // ---- A panel -> LDS (as igemm_panel_kernel)
        const __amdgpu_buffer_rsrc_t ra = make_rsrc(uniform_ptr(p.src0), (unsigned)((size_t)p.M * p.c0 * 2));
        constexpr int RG = BM / 8, PIECES = RG * NKB;
        for (int pc = wave; pc < PIECES; pc += 8) {
            const int kb = pc / RG, rg = pc - kb * RG;
            const int row = rg * 8 + lrow, m = m0 + row;
            const int ch = kb * 64 + ((lslot ^ ((row >> 1) & 7)) << 3);
            const unsigned off = m < p.M ? (unsigned)(2 * (m * p.c0 + ch)) : kOOB;
            dma_piece(ra, smem + kb * BLK + rg * 1024, off);
        }
    }
    const int nblk = p.cout >> 5, stride = 8 * nsplit;
    const int j0 = split * 8 + wave;
    char* ring = smem + A_BYTES + wave * 2 * BSLOT;
    const char* u_wt = uniform_ptr(p.wt);
    const unsigned wbytes = (unsigned)((size_t)p.cout * p.kpad * 2);
    unsigned boffq[4];   // piece q: weight row 8 q + lrow of the block, swizzled 16-B chunk
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = 8 * q + lrow;
        boffq[q] = (unsigned)(2 * (row * p.kpad + ((lslot ^ ((row >> 1) & 7)) << 3)));
    }
    auto bdma = [&](int j, int t, int sl) __attribute__((always_inline)) {
        const unsigned base = 2u * (unsigned)(32 * j * p.kpad + 64 * t);
        const __amdgpu_buffer_rsrc_t rb = make_rsrc(u_wt + base, wbytes - base);
#pragma unroll
        for (int q = 0; q < 4; ++q) dma_piece(rb, ring + sl * BSLOT + q * 1024, boffq[q]);
    };
    const int jfirst = j0 < nblk ? j0 : 0;
    bdma(jfirst, 0, 0);
    const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias, p.bias ? (unsigned)(p.cout * 4) : 0u);
    float4 bv[2];   // bias of the next column block: its accumulators start from it
    auto bload = [&](int j) __attribute__((always_inline)) {
        const int lc = 32 * j + 4 * (lane >> 4);
#pragma unroll
        for (int a = 0; a < 2; ++a)
            bv[a] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rbias, 4 * (lc + 16 * a), 0, 0));
    };
    bload(jfirst);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    C2D_PSTAMP(1);
    if constexpr (LNF) {
        panel_ln_inplace<NKB>(smem, wave, lane, p.pro_eps);
        __syncthreads();
    }
    if (j0 >= nblk) return;   // wave-uniform; no barrier follows
    // waves 4-7 (the second wave of each SIMD) start `stagger` x 2048 cycles late, so that on every
    // SIMD one wave's epilogue (VALU, stores) runs beside its partner's K loop (MFMA) instead of
    // every wave of the chip storing at once
    if (wave >= 4)
        for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(32);
    if (C2D_TUNE_PANEL_PRIO && wave >= 4) __builtin_amdgcn_s_setprio(1);   // static priority, waves 4-7 (A/B)
    int sbi = 0;   // stamp block index (diagnostic builds)
    (void)sbi;

    int fa0[2], fbo[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        fa0[h] = lds_off(lane & 15, h * 4 + (lane >> 4));
#pragma unroll
        for (int a = 0; a < 2; ++a) fbo[a][h] = lds_off(16 * a + (lane & 15), h * 4 + (lane >> 4));
    }
    const __amdgpu_buffer_rsrc_t rres = make_rsrc(p.resid, p.resid ? (unsigned)((size_t)p.M * p.resid_ld * 2) : 0u);
    f16x8 fa[2][8];
    auto aread = [&](int ks, f16x8 (&dst)[8]) {
        const char* S = smem + (ks >> 1) * BLK + fa0[ks & 1];
#pragma unroll
        for (int b = 0; b < 8; ++b) dst[b] = *reinterpret_cast<const f16x8*>(S + b * 2048);
    };
    aread(0, fa[0]);
    int par = 0;   // ring slot of the block's step 0 (5 steps per block: it alternates)
    // CARRY (GEGLU, C2D_TUNE_PANEL_CARRY): a block's epilogue runs inside the next block's K loop,
    // one 16-row tile per K half-step (steps 0-7 of 10) among that step's MFMAs, from the previous
    // block's accumulators kept in registers; the last block's is flushed after the loop.  Every
    // carried half-step issues one store, so the counted waits of the steps after it allow one more
    constexpr bool CARRY = C2D_TUNE_PANEL_CARRY && EPI == PE_GEGLU;
    f32x4 accp[2][8];
    int jprev = 0;
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(p.out, (unsigned)((size_t)p.M * p.out_ld * 2));
    auto carry_row = [&](int b) __attribute__((always_inline)) {
        const int m = m0 + b * 16 + (lane & 15);
        const unsigned off = m < p.M ? (unsigned)(2 * (m * p.out_ld + 16 * jprev + 4 * (lane >> 4))) : kOOB;
        f16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (f16)(accp[0][b][r] * gelu_sig(accp[1][b][r]));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), rout, off, 0, 0);
    };
    auto block = [&](int j, bool first) __attribute__((always_inline)) {
        C2D_PSTAMP(2 + 8 * sbi);
        const int jn = j + stride < nblk ? j + stride : j;
        f32x4 acc[2][8];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 8; ++b) acc[a][b] = (f32x4){bv[a].x, bv[a].y, bv[a].z, bv[a].w};
        f16x4 rv[8][2];
#pragma unroll
        for (int t = 0; t < NKB; ++t) {
            if (t == NKB - 1) {   // epilogue operands and the next block's bias, ahead of its first weights
                const int lc = 32 * j + 4 * (lane >> 4);
                bload(jn);
                if constexpr (EPI == PE_RESID) {
#pragma unroll
                    for (int b = 0; b < 8; ++b) {
                        const int m = m0 + b * 16 + (lane & 15);
                        const unsigned ro = (unsigned)(2 * ((m < p.M ? m : 0) * p.resid_ld + lc));
#pragma unroll
                        for (int a = 0; a < 2; ++a)
                            rv[b][a] = __builtin_bit_cast(f16x4, __builtin_amdgcn_raw_buffer_load_b64(rres, ro + 32 * a, 0, 0));
                    }
                }
                bdma(jn, 0, (par + NKB) & 1);
                if (CARRY && !first) panel_wait_vm<4 + NRES + 2>();
                else panel_wait_vm<4 + NRES>();
            } else {
                bdma(j, t + 1, (par + t + 1) & 1);
                if (CARRY) {
                    if (t > 0 && !first) panel_wait_vm<4 + 2>();
                    else panel_wait_vm<4>();
                } else if (t == 0 && !first) panel_wait_vm<4 + NST>();
                else panel_wait_vm<4>();
            }
            C2D_PSTAMP(3 + 8 * sbi + t);
            const char* B = ring + ((par + t) & 1) * BSLOT;
            f16x8 fb[2][2];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int a = 0; a < 2; ++a) fb[h][a] = *reinterpret_cast<const f16x8*>(B + fbo[a][h]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ks = 2 * t + h;
                aread(ks + 1 < 2 * NKB ? ks + 1 : 0, fa[(ks + 1) & 1]);
                if (CARRY && !first && ks < 8) carry_row(ks);
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    acc[0][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[h][0], fa[ks & 1][b], acc[0][b], 0, 0, 0);
                    acc[1][b] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[h][1], fa[ks & 1][b], acc[1][b], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        C2D_PSTAMP(8 + 8 * sbi);
        if constexpr (CARRY) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 8; ++b) accp[a][b] = acc[a][b];
            jprev = j;
        } else {
            panel_epilogue<EPI>(p, acc, rv, m0, 32 * j, lane);
        }
        C2D_PSTAMP(9 + 8 * sbi);
        ++sbi;
        par ^= 1;
    };
    block(j0, true);
    for (int j = j0 + stride; j < nblk; j += stride) block(j, false);
    if constexpr (CARRY) {
#pragma unroll
        for (int b = 0; b < 8; ++b) carry_row(b);
    }
    panel_wait_vm<0>();   // the last block's look-ahead pieces land before the workgroup's LDS is released
}

// column blocks shared out over nsplit workgroups per panel when the panels alone leave CUs idle
static int panel_nsplit(int M, int cout) {
    const int panels = (M + kPanelRows - 1) / kPanelRows, nblk = cout >> 5;
    int ns = (256 + panels - 1) / panels;
    const int maxs = (nblk + 7) / 8;
    return ns < 1 ? 1 : (ns > maxs ? maxs : ns);
}

template <int NK32, int EPI, bool LNF = false>
static void launch_panel(IgemmParams& p, hipStream_t s) {
    constexpr int smem = NK32 / 2 * kPanelRows * 128;
    static_assert(smem <= 160 * 1024, "A panel too large");
    ensure_lds<igemm_panel_kernel<NK32, 5, EPI, LNF>>(smem);
    const int ns = panel_nsplit(p.M, p.cout);
    const int grid = (p.M + kPanelRows - 1) / kPanelRows * ns;
    hipLaunchKernelGGL((igemm_panel_kernel<NK32, 5, EPI, LNF>), dim3(grid), dim3(512), smem, s, p, ns);
}

template <int NK32>
static void launch_panel_epi(IgemmParams& p, hipStream_t s) {
    if (p.act == C2D_ACT_GEGLU) launch_panel<NK32, PE_GEGLU>(p, s);
    else if (p.resid) launch_panel<NK32, PE_RESID>(p, s);
    else launch_panel<NK32, PE_PLAIN>(p, s);
}

#if defined(C2D_PANEL_STAMP) && C2D_PART(4)
}  // namespace c2d
// diagnostic variant only (not in c2d.h): copy the stamps of the last stamped launch to host memory
extern "C" int c2d_debug_panel_stamps(unsigned long long* host, int n) {
    if (n > 8 * c2d::kPanelStampPer) n = 8 * c2d::kPanelStampPer;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(c2d::g_panel_stamps), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -4;
}
namespace c2d {
#endif

template <int EPI, bool LNF = false>
static void launch_panel_dma(IgemmParams& p, hipStream_t s) {
    constexpr int smem = 5 * kPanelRows * 128 + 8 * 2 * 32 * 128;   // 80 + 64 KiB
    ensure_lds<igemm_panel_dma_kernel<EPI, LNF>>(smem);
    const int ns = panel_nsplit(p.M, p.cout);
    const int grid = (p.M + kPanelRows - 1) / kPanelRows * ns;
    hipLaunchKernelGGL((igemm_panel_dma_kernel<EPI, LNF>), dim3(grid), dim3(512), smem, s, p, ns,
                       tuning().panel_stagger);
}

// K = 320 / 640 only (panel_eligible: also no GEGLU + residual); 32-bit offsets into A (dma_eligible).
// A folded LayerNorm (C2D_PRO_LNFOLD) takes the LDS-DMA form at K = 320.
static void run_panel(IgemmParams& p, hipStream_t s) {
    if (p.pro == C2D_PRO_LNFOLD) {
        if (p.kpad == 320) {
            if (p.act == C2D_ACT_GEGLU) launch_panel_dma<PE_GEGLU, true>(p, s);
            else launch_panel_dma<PE_PLAIN, true>(p, s);
        } else {
            if (p.act == C2D_ACT_GEGLU) launch_panel<20, PE_GEGLU, true>(p, s);
            else launch_panel<20, PE_PLAIN, true>(p, s);
        }
    } else if (p.kpad == 320 && !tuning().panel_regb) {
        if (p.act == C2D_ACT_GEGLU) launch_panel_dma<PE_GEGLU>(p, s);
        else if (p.resid) launch_panel_dma<PE_RESID>(p, s);
        else launch_panel_dma<PE_PLAIN>(p, s);
    } else if (p.kpad == 320) {
        launch_panel_epi<10>(p, s);
    } else {
        launch_panel_epi<20>(p, s);
    }
}

}  // namespace c2d
