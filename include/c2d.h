/*
 * c2d.h — C ABI of libc2d_hip.so, the MI355X (gfx950) kernels behind the
 * audio-conditioned SD1.5 denoise step and the CLAP HTSAT audio tower.
 *
 * Conventions:
 *   - Every buffer is device memory owned by the caller; the library never
 *     allocates.  Activations are NHWC / row-major fp16, statistics fp32.
 *   - Every entry point is stream-ordered on the hipStream_t passed in (passed
 *     as void* so that this header needs no HIP include) and is safe to capture
 *     into a hipGraph: no allocation, no synchronisation, no host reads.
 *   - Return 0 on success, a negative C2D_E_* code on a shape / alignment /
 *     argument error (nothing is launched then), C2D_E_HIP when the launch
 *     itself failed (hipError_t from c2d_last_hip_error(), thread-local).
 *
 * Which reference interface each entry point replaces is cited per function
 * (reference = youdie006/CLAP2Diffusion @ /root/reference, plus the
 * third-party diffusers==0.23.1 / transformers ops it glues together).
 */
#ifndef C2D_H
#define C2D_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define C2D_OK 0
#define C2D_E_ARG (-1)       /* null pointer / bad enum                        */
#define C2D_E_SHAPE (-2)     /* unsupported or inconsistent shape              */
#define C2D_E_ALIGN (-3)     /* pointer / leading dimension not 16-B aligned   */
#define C2D_E_HIP (-4)       /* kernel launch failed, see c2d_last_hip_error() */

/* prologue applied to every in-bounds A element before the MMA */
#define C2D_PRO_NONE 0
#define C2D_PRO_GN 1         /* y = x*scale[n][c] + shift[n][c]  (GroupNorm affine, folded) */
#define C2D_PRO_LN 2         /* y = (x-mean[m])*rstd[m]*gamma[c] + beta[c]                  */
#define C2D_PRO_SILU 3       /* y = silu(x)                                                 */
/* LayerNorm folded into a 1x1 GEMM whose K is the whole row (one source, c0 = kpad = 320 / 640,
 * the panel GEMM): the kernel normalises each row of the A panel it holds in LDS in place,
 * (x - mean) * rstd rounded to fp16 (eps = pro_eps), and runs the GEMM on it -- the
 * LayerNorm(gamma, beta) -> Linear(W, b) pair with weight = W diag(gamma) (fp16) and
 * bias = b + W beta (fp32).  pro_a / pro_b unused.  Act none or GEGLU, no residual / temb.
 * Shapes the panel GEMM does not take: C2D_E_SHAPE.
 * Replaces BasicTransformerBlock norm1 -> to_q/k/v and norm3 -> GEGLU (diffusers attention.py,
 * reached from reference models/audio_attention_processor.py:115). */
#define C2D_PRO_LNFOLD 4

/* activation applied after the bias in the epilogue */
#define C2D_ACT_NONE 0
#define C2D_ACT_GEGLU 1      /* weight rows interleaved in 16-row h/g blocks; out = h*gelu(g) */
#define C2D_ACT_GELU 2       /* exact erf GELU */
#define C2D_ACT_RELU 3
#define C2D_ACT_SILU 4
#define C2D_ACT_QUICK_GELU 5 /* x * sigmoid(1.702 x) (CLIP text MLP, transformers ACT2FN["quick_gelu"]) */

/*
 * Implicit-GEMM convolution / linear layer on MFMA (v_mfma_f32_16x16x32_f16).
 *   out[m, j] = act( sum_k A[m,k] * W[j,k] + bias[j] ) + temb[n(m), j] + resid[m, j]
 * where A is the (virtual) im2col of the NHWC input after the prologue, with
 * K ordered (ky, kx, cin) and W packed as [cout][kpad] (kpad = K rounded up to 64,
 * zero filled).  Input channels may come from two sources (skip concat:
 * channels [0,c0) from src0, [c0,c0+c1) from src1) without materialising the
 * concatenation.  ksize 1 = linear / 1x1 conv; ksize 3 = 3x3 conv with pad 1,
 * stride 1 or 2, optionally reading a nearest-x2-upsampled view of the input.
 *
 * Replaces (diffusers 0.23.1): ResnetBlock2D.norm1/2+SiLU+conv1/conv2+temb add+
 * shortcut, Downsample2D/Upsample2D convs, conv_in/conv_out, Transformer2DModel
 * proj_in/proj_out, Attention.to_q/k/v/to_out, GEGLU+FeedForward, TimestepEmbedding;
 * reached from reference models/audio_attention_processor.py:115-135 (to_q/to_k/
 * to_v/to_out) and the UNet the processor plugs into.
 * Also transformers ClapAudioLayer / PatchMerging / ClapProjectionLayer linears
 * (modeling_clap.py:323-478, 680-717, 905-921) via models/audio_encoder.py:171.
 */
typedef struct c2d_conv_desc {
    const void* src0;        /* fp16 NHWC [n][h][w][c0]                                   */
    const void* src1;        /* fp16 NHWC [n][h][w][c1] or NULL                           */
    int c0, c1;              /* channels per source (c1 = 0 without a second source)      */
    int n, h, w;             /* input batch and spatial size (source resolution)          */
    int oh, ow;              /* output spatial size                                       */
    int ksize;               /* 1 or 3                                                    */
    int stride;              /* 1 or 2 (3x3 only)                                         */
    int up;                  /* 1: conv reads nearest-x2 upsampled input (3x3, stride 1)  */
    const void* weight;      /* fp16 [cout][kpad]                                         */
    int cout;                /* output columns (packed rows; GEGLU: 2x the output width)  */
    int kpad;                /* packed K, multiple of 64, >= ksize*ksize*(c0+c1)          */
    int pro;                 /* C2D_PRO_*                                                 */
    int pro_silu;            /* GN prologue: apply SiLU after the affine                  */
    const float* pro_a;      /* GN: scale [n][c0+c1]   LN: (mean,rstd) [m][2]             */
    const float* pro_b;      /* GN: shift [n][c0+c1]   LN: unused                         */
    const float* gamma;      /* LN gamma [c]                                              */
    const float* beta;       /* LN beta  [c]                                              */
    const float* bias;       /* fp32 [cout] or NULL                                       */
    int act;                 /* C2D_ACT_*                                                 */
    const void* temb;        /* fp16 [n][temb_ld] added per (image, column) or NULL       */
    int temb_ld;
    const void* resid;       /* fp16 [m][resid_ld] added after the activation or NULL     */
    int resid_ld;
    void* out;               /* fp16 [m][out_ld]                                          */
    int out_ld;
    void* ws;                /* optional split-K workspace (16-B aligned) or NULL         */
    size_t ws_bytes;         /* its size; below c2d_conv2d_igemm_workspace_size(): no split */
    int src_pad;             /* 1: src0 is zero-bordered, [n][h+2][w+2][c0] (c2d_groupnorm_pad):
                                3x3, stride 1, one source, output h x w; tile 42 (the row-ring
                                conv) runs it at w = 64, every other tile as a valid 3x3.
                                No prologue (pro must be C2D_PRO_NONE, else C2D_E_ARG): the
                                border is read as data, so a GN / LN / SiLU would turn it into
                                act(shift) instead of the zero padding torch applies        */
    float pro_eps;           /* C2D_PRO_LNFOLD: the LayerNorm eps                         */
    /* r6: GroupNorm moments of the output, emitted by the producer (NULL = none).  When set,
       the conv also writes, for every block of c2d_conv2d_gn_rows(d) output rows of one image
       and every one of gn_groups channel groups, the fp32 pair {mean, M2} (M2 = sum of squared
       deviations from that mean) of the fp16 values it stores: layout
       [n][oh * ow / rows][gn_groups][2].  c2d_groupnorm_moments then normalises the output
       without re-reading it for statistics.  Only where c2d_conv2d_gn_rows(d) > 0, else
       C2D_E_SHAPE.  Callers built against the r5 header (no such fields) must not be mixed with
       this library: the descriptor grew (c2d_version "r6").                              */
    void* gn_mom;
    int gn_groups;           /* channel groups of the moments (cout % gn_groups == 0)     */
} c2d_conv_desc;

int c2d_conv2d_igemm(const c2d_conv_desc* d, void* stream);

/*
 * Bytes of split-K workspace c2d_conv2d_igemm would use for this descriptor
 * (0 = the shape fills the chip without splitting K; sized for fp32 partials).  A one-slice
 * plan can still ask for some: when its grid is whole rounds of the chip plus at most a quarter
 * round (c5's level-0 convs: 288 tiles on 256 CUs), the last images run as a second launch on
 * their own plan, which may split K (c2d_conv2d_igemm_plan reports the first launch's plan).
 * Under-filled GEMMs (the 16x16 / 8x8 UNet levels: 80-160 output tiles on 256 CUs)
 * split K across blocks into [split][m][cout] slabs of partial sums that a second,
 * stream-ordered kernel adds in fp32 in fixed order before the epilogue
 * (deterministic; no atomics).  Partials are fp32 (the MFMA sum of the K slice, unrounded):
 * K slices whose partials cancel -- each far above the output, e.g. beyond the fp16 range
 * while the output fits -- combine to the same result as the single-pass GEMM
 * (tests/test_kernels_gpu.py::test_split_k_cancelling_partials_beyond_fp16).
 * A variant build with -DC2D_TUNE_SPLITK_F16=1 (A/B only) stores them rounded to fp16: half the
 * slab bytes, but a partial beyond +-65504 becomes inf and cancelling partials lose
 * 2^-11 of their own magnitude.
 */
size_t c2d_conv2d_igemm_workspace_size(const c2d_conv_desc* d);

/*
 * The kernel plan c2d_conv2d_igemm would run for this descriptor (no launch, no device
 * access): tile_id = the LDS-DMA tile configuration (0 = the register-staged kernel of
 * descriptors with a prologue / upsampled view), ksplit = K slices (1 = no split-K;
 * reflects d->ws / d->ws_bytes as the launch would).  Lets callers and the per-tile
 * parity test (tests/test_kernels_gpu.py) see which kernel ran; c2d_set_plan_override
 * forces a plan (tuning and tests only).
 */
int c2d_conv2d_igemm_plan(const c2d_conv_desc* d, int* tile_id, int* ksplit);

/*
 * Rows per GroupNorm-moment block if c2d_conv2d_igemm can emit the moments of this descriptor's
 * output (c2d_conv_desc::gn_mom, gn_groups), 0 if not.  One-slice plans: the row-ring 3x3 tiles
 * (42: 256 rows, 43 / 44: 128) and the 256 x 320 ping-pong tile 40 (256) with a residual or a time
 * embedding (their workgroup-image epilogue computes each column's shifted moments over the tile from
 * the stored fp16 values and folds them per group in a fixed order); split-K plans: the combine kernel
 * (16-row blocks, exact per-thread moments merged in a fixed order).  Always act none, no
 * quantisation-tail split, 16-B aligned outputs, 320 % (cout / gn_groups) == 0 and cout % 320 == 0.
 * The SD1.5 UNet's ResnetBlock2D conv1 (+ temb) -> norm2, conv2 (+ residual) -> the next norm, and the
 * Transformer2DModel output / downsampler -> the next resnet's norm1.
 */
int c2d_conv2d_gn_rows(const c2d_conv_desc* d);

/*
 * Test / tuning hook: force the LDS-DMA tile configuration (tile_id, one of the ids
 * c2d_conv2d_igemm_plan reports) and the K split (ksplit; 0 = the planner's) of every
 * later eligible c2d_conv2d_igemm call in the process; c2d_set_plan_override(0, 0)
 * restores the planner.  Process-wide (atomic), set explicitly: the library reads no
 * environment variable at all (its tuning constants are compile-time, csrc/common.h).  C2D_E_ARG for negative values or ksplit > 64.
 */
int c2d_set_plan_override(int tile_id, int ksplit);

/* The override c2d_set_plan_override last set ((0, 0) = the planner); lets a scoped
 * override restore the enclosing one.  C2D_E_ARG for NULL pointers. */
int c2d_get_plan_override(int* tile_id, int* ksplit);

/*
 * GroupNorm statistics folded with the affine into per-(image, channel) scale /
 * shift tables consumed by the C2D_PRO_GN prologue:
 *   scale[n][c] = gamma[c]*rstd[n,g(c)], shift[n][c] = beta[c] - mean[n,g(c)]*scale[n][c]
 * Input may be a two-source channel concat (GroupNorm over the concatenation,
 * groups may straddle the seam).  ws: fp32 workspace of
 * c2d_groupnorm_workspace_size(n, c, hw) bytes holding per-block partial moments
 * (plain stores, fixed-order reduction: deterministic, no atomics, no memset).
 * Limits: (c0 + c1) / groups <= 256 channels per group, channels multiples of 8.
 * Replaces torch.nn.GroupNorm in ResnetBlock2D.norm1/norm2 (eps 1e-5) and
 * Transformer2DModel.norm (eps 1e-6), diffusers 0.23.1.
 */
size_t c2d_groupnorm_workspace_size(int n, int c, int hw);
int c2d_groupnorm_stats(const void* src0, const void* src1, int c0, int c1, int n, int hw,
                        int groups, float eps, const float* gamma, const float* beta,
                        float* scale, float* shift, void* ws, void* stream);

/*
 * GroupNorm apply with the folded tables: out[m][c] = act(x[m][c]*scale[n][c] + shift[n][c]),
 * act = SiLU when silu != 0; the input may be a two-source concat, the output is the
 * concatenation (fp16 [n*hw][c0+c1]).  The UNet materialises each normalised tensor once
 * (HBM-bound) instead of re-normalising it in every 3x3 tap / N-tile of the consuming GEMM.
 * Limits: c0 + c1 <= 4096.
 */
int c2d_groupnorm_apply(const void* src0, const void* src1, int c0, int c1, int n, int hw,
                        const float* scale, const float* shift, int silu, void* out, void* stream);

/*
 * act(GroupNorm(cat[src0, src1])) in one call -- what HGroupNorm.apply (the
 * ResnetBlock2D.norm1/norm2 + SiLU, Transformer2DModel.norm, conv_norm_out and VAE
 * norms) needs.  Small images (hw <= 256 pixels) run a single kernel: one
 * workgroup per (image, chunk of whole groups) computes the statistics, folds them in
 * a fixed order and applies in a second pass over the L2 / MALL-resident slab.
 * Larger ones run two kernels: per-block partial moments folded per group (ws >=
 * c2d_groupnorm_run_workspace_size(n, c0+c1, hw, groups) bytes, 16-B aligned; the size is
 * 0 -- ws may be NULL -- when the single kernel runs), then an apply kernel whose
 * workgroups fold an image's group partials in a fixed order themselves (no separate
 * finalize launch; up to 256 groups, else c2d_groupnorm_stats + c2d_groupnorm_apply).
 * Deterministic either way.
 */
size_t c2d_groupnorm_run_workspace_size(int n, int c, int hw, int groups);
int c2d_groupnorm(const void* src0, const void* src1, int c0, int c1, int n, int hw, int groups,
                  float eps, const float* gamma, const float* beta, int silu, void* out,
                  void* ws, size_t ws_bytes, void* stream);

/*
 * c2d_groupnorm writing the zero-bordered layout out[n][h + 2][w + 2][c0 + c1] (border
 * pixels 0, interior = act(GroupNorm(cat[src0, src1]))): the input of a 3x3 conv with
 * c2d_conv_desc::src_pad = 1 (ResnetBlock2D.norm1/norm2 + SiLU feeding conv1/conv2), whose
 * taps then need no halo masks and which tile 42 (the row-ring conv) stages once per channel
 * block.  Statistics as c2d_groupnorm_stats (deterministic); ws >=
 * c2d_groupnorm_pad_workspace_size(n, c0 + c1, h, w) bytes, 16-B aligned.
 */
size_t c2d_groupnorm_pad_workspace_size(int n, int c, int h, int w);
int c2d_groupnorm_pad(const void* src0, const void* src1, int c0, int c1, int n, int h, int w, int groups,
                      float eps, const float* gamma, const float* beta, int silu, void* out, void* ws,
                      size_t ws_bytes, void* stream);

/*
 * act(GroupNorm(src)) from moments its producer emitted (c2d_conv_desc::gn_mom): mom holds fp32
 * {mean, M2} per (image, block of `rows` pixels, group), [n][hw / rows][groups][2].  Every apply
 * workgroup of image n merges its image's blocks per group (equal block counts: fp64 sums of the
 * blocks' M2 and of their means shifted by block 0's, fixed order: deterministic) and applies; one
 * launch, no statistics pass over src.  pw = 0: plain output
 * [n][hw][c]; pw = w + 2 (h = hw / w): the zero-bordered layout of c2d_groupnorm_pad.  One source
 * (c <= 4096, multiple of 8), groups <= 256, hw % rows == 0.
 */
int c2d_groupnorm_moments(const void* src, int c, int n, int hw, int groups, float eps, const float* gamma,
                          const float* beta, int silu, const float* mom, int rows, int pw, void* out,
                          void* stream);

/*
 * LayerNorm over rows of a row-major fp16 [m][c] matrix (leading dim ld).
 * c2d_layernorm_stats writes (mean, rstd) [m][2] for the C2D_PRO_LN prologue;
 * c2d_layernorm writes the normalised fp16 rows (out_ld) with gamma/beta.
 * Replaces nn.LayerNorm in BasicTransformerBlock.norm1/2/3 (diffusers) and
 * ClapAudioPatchEmbed.norm / ClapAudioLayer.layernorm_before/after /
 * ClapAudioEncoder.norm (modeling_clap.py:233-321, 504-621, 720-902).
 */
int c2d_layernorm_stats(const void* x, int m, int c, int ld, float eps, float* stats, void* stream);
int c2d_layernorm(const void* x, int m, int c, int ld, float eps, const float* gamma,
                  const float* beta, void* out, int out_ld, void* stream);

/*
 * Flash-style attention forward, fp16 in/out, fp32 softmax, online max.
 *   O[b, i, h*d:(h+1)*d] = softmax_j( Q_bhi . K_bhj * scale ) V_bhj
 * Q/K/V/O are row-major token matrices with leading dims (elements); head h
 * occupies columns [h*d, (h+1)*d) of each.  d in {40, 64, 80, 160}.
 * lk may be any length (tail keys masked).  K/V batch index = b / kv_div
 * (kv_div = 1 normally).
 * Replaces the attention math of reference AudioAttnProcessor.__call__
 * (models/audio_attention_processor.py:114-135: head_to_batch_dim,
 * get_attention_scores, bmm, batch_to_head_dim) and AttnProcessor2_0 (attn1).
 */
int c2d_attention_fwd(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                      void* o, int ldo, int batch, int heads, int lq, int lk, int d,
                      float scale, int kv_div, void* stream);

/*
 * c2d_attention_fwd with an additive per-key score bias (the attention_mask of the
 * processor API, reference models/audio_attention_processor.py:48,129 -> diffusers
 * Attention.get_attention_scores, baddbmm(mask, q, k^T, beta=1, alpha=scale), in the
 * key-padding form diffusers builds from encoder_attention_mask, (1 - keep) * -10000):
 *   S[b, h, i, j] = Q.K * scale + key_bias[b * bias_ld_batch + h * bias_ld_head + j]
 * fp32 bias, natural-log units; strides 0 broadcast over images / heads.  key_bias NULL
 * is exactly c2d_attention_fwd.  Bias entries may be -inf (SDPA-style boolean masks) or
 * finfo(float).min: a row with at least one finite score is exact; a row whose every
 * score is -inf comes out NaN, as torch's softmax of such a row does (the reference
 * path, get_attention_scores + softmax); a row of finfo.min entries comes out as the
 * uniform average of V, as torch's does.
 */
int c2d_attention_fwd_bias(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                           void* o, int ldo, int batch, int heads, int lq, int lk, int d, float scale,
                           int kv_div, const float* key_bias, int bias_ld_batch, int bias_ld_head,
                           void* stream);

/*
 * The general form: any attention_mask broadcastable to [batch*heads, lq, lk], as the
 * reference processor hands it unchanged to get_attention_scores
 * (models/audio_attention_processor.py:129; diffusers baddbmm(mask, q, k^T, beta=1,
 * alpha=scale)), including masks that vary over queries:
 *   S[b, h, i, j] = Q.K * scale + bias[b * bias_ld_batch + h * bias_ld_head + i * bias_ld_query + j]
 * Strides 0 broadcast.  bias_ld_query = 0 is c2d_attention_fwd_bias; same -inf rules.
 */
int c2d_attention_fwd_mask(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                           void* o, int ldo, int batch, int heads, int lq, int lk, int d, float scale,
                           int kv_div, const float* bias, int bias_ld_batch, int bias_ld_head,
                           int bias_ld_query, void* stream);

/*
 * Swin window attention of the HTSAT tower: tokens gathered through row_map
 * (window w, token t -> row of the [B*H*W] token matrix; encodes the cyclic
 * shift + window partition), 64-token windows, head dim 24, relative-position
 * bias [heads][64][64] plus an optional shift mask [n_mask][64][64] indexed by
 * window % n_mask, output scattered back through row_map.
 * Replaces ClapAudioSelfAttention.forward + window_partition/window_reverse/
 * torch.roll (transformers modeling_clap.py:64-100, 323-414, 558-621).
 */
int c2d_window_attention(const void* qkv, int ld_qkv, const int* row_map, int n_windows,
                         int heads, int d, const float* bias, const float* mask, int n_mask,
                         void* out, int ldo, void* stream);

/*
 * HTSAT input stage: BatchNorm2d over mel bins (eval affine), bicubic time
 * resize 1001->1024 (align_corners), fold to 256x256 and cut 4x4 patches:
 * out fp16 [b*4096][64] (16 used columns, zero pad).  mel fp32 [b][t][64].
 * Replaces ClapAudioEncoder.forward:batch_norm + reshape_mel2img and the im2col
 * of ClapAudioPatchEmbed.proj (modeling_clap.py:761-798, 814-828, 224-321).
 */
int c2d_htsat_mel_patches(const float* mel, int b, int t, const float* bn_scale,
                          const float* bn_shift, void* out, void* stream);

/* Swin PatchMerging gather: [b][h][w][c] -> [b][h/2*w/2][4c] in the
 * (r0c0, r1c0, r0c1, r1c1) order of ClapAudioPatchMerging.forward (modeling_clap.py:700-717). */
int c2d_patch_merge_gather(const void* x, int b, int h, int w, int c, void* out, void* stream);

/* Row mean over groups of `rows` consecutive rows: out fp32 [b][c] = mean_r x[b*rows+r][c]
 * (ClapAudioEncoder avgpool over the final 64 tokens, modeling_clap.py:880-896). */
int c2d_row_mean(const void* x, int b, int rows, int c, int ld, float* out, void* stream);

/* Row-wise L2 normalise fp32 [m][c] in place (F.normalize, modeling_clap.py:1533). */
int c2d_l2_normalize(float* x, int m, int c, void* stream);

/* Short-sequence attention, l <= 128 keys = queries, d = 64, optional causal mask
 * (key j visible to query i iff j <= i): the CLIP ViT-L/14 text tower's self-attention
 * (transformers CLIPAttention + its causal mask, the encoder_hidden_states producer of
 * the SD1.5 pipeline the reference drives).  Row layout as
 * c2d_attention_fwd: head h of token t of image b at [b*l + t][h*d ..]. */
int c2d_attention_small(const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* o,
                        int ldo, int batch, int heads, int l, int d, float scale, int causal, void* stream);

/* CLAP log-mel front end: the reference's audio composition -- CLAPAudioEncoder.preprocess_audio
 * (models/audio_encoder.py:121-129: zero-pad to max_len = 10 s x 48 kHz samples, or keep the
 * first max_len) then transformers ClapFeatureExtractor on that exact-length clip
 * (feature_extraction_clap.py _get_input_mel: no repeat-pad / crop at exact length;
 * audio_utils.spectrogram with a periodic Hann window, centre reflect pad, power 2, mel
 * filters, dB; models/audio_encoder.py:163-167).  wave: fp32 clips concatenated, clip i at
 * wave + offsets[i] with lengths[i] samples; lengths are clamped to [0, max_len] on the
 * device (longer -> first max_len samples, 0 -> silence = -100 dB), so no length can fault.
 * window fp32 [n_fft]; mel_filters fp32 [n_mels][n_fft/2+1]; filter_range int [n_mels][2] =
 * the non-zero bin range [lo, hi) of each filter.  out fp32 [b][1 + max_len/hop][n_mels].
 * n_fft must be 1024. */
int c2d_clap_log_mel(const float* wave, const long long* offsets, const int* lengths, int b, int max_len,
                     int n_fft, int hop, const float* window, const float* mel_filters,
                     const int* filter_range, int n_mels, float* out, void* stream);

/* Weight prepack for c2d_conv2d_igemm: fp32 [cout][cin][ksize][ksize] (PyTorch layout;
 * ksize 1 for a Linear [cout][cin]) -> fp16 [cout][kpad] with K ordered (ky, kx, channel)
 * over cin_pad >= cin channels, zero-filled past cin and past ksize^2 * cin_pad;
 * kpad % 64 == 0.  Replaces the layout work diffusers / transformers never do (their
 * convs run NCHW through cuDNN / MIOpen); one-time, at checkpoint load. */
int c2d_pack_weights(const float* w, int cout, int cin, int ksize, int cin_pad, int kpad, void* out,
                     void* stream);

/* Row softmax fp16 [rows][cols] (leading dims ld / ldo, elements) -> fp16, fp32 math;
 * cols % 8 == 0, cols <= 16384, 16-B aligned rows.  The score normalisation of the
 * materialised single-head attention in the VAE decoder's mid block (diffusers
 * Attention(512, heads=1) inside UNetMidBlock2D of AutoencoderKL; diffusers 0.23.1 is
 * absent from the reference tree, which loads it through scripts/inference.py:30-33).
 * May run in place (out == x, ldo == ld). */
int c2d_softmax_rows(const void* x, int rows, int cols, int ld, void* out, int ldo, void* stream);

/*
 * Sinusoidal timestep embedding of diffusers get_timestep_embedding with
 * flip_sin_to_cos=True, downscale_freq_shift=0: out fp16 [n][dim] = [cos, sin](t*f_i).
 * t read from device memory: t_table[*step_index] (so a captured graph can be
 * replayed across DDIM steps), broadcast to n rows.
 */
int c2d_timestep_embedding(const float* t_table, const int* step_index, int n, int dim,
                           void* out, void* stream);

/*
 * Fused classifier-free guidance + DDIM (eta = 0) update, fp32 latents:
 *   e = eps_u + g*(eps_c - eps_u); x0 = (x - sqrt(1-a_t) e)/sqrt(a_t);
 *   x <- sqrt(a_prev) x0 + sqrt(1 - a_prev) e
 * eps fp16 NHWC [2b][hw][4] (uncond rows first), x fp32 NCHW [b][4][hw] in place.
 * coef fp32 [steps][2] = (a_t, a_prev) per step, read at *step_index; when
 * advance != 0 the kernel increments *step_index after use (last block).
 * Replaces the pipeline CFG combine + DDIMScheduler.step (diffusers 0.23.1).
 */
int c2d_cfg_ddim_step(const void* eps, float* x, int b, int c, int hw, float guidance,
                      const float* coef, int* step_index, int advance, void* stream);

/* NCHW fp32 [n][c][hw] -> NHWC fp16 [2*n or n][hw][cpad] (zero-padded channels), optional
 * duplication for the CFG pair (dup=1 writes rows n..2n-1 again). */
int c2d_latent_to_nhwc(const float* x, int n, int c, int hw, int cpad, int dup, void* out,
                       void* stream);

/* Nearest-neighbour x2 upsample of NHWC fp16 [n, h, w, c] -> [n, 2h, 2w, c], c % 8 == 0.
 * Replaces F.interpolate(scale_factor=2.0, mode="nearest") in diffusers Upsample2D
 * (the UNet up path and the VAE decoder). */
int c2d_upsample_nearest2x(const void* x, int n, int h, int w, int c, void* out, void* stream);

/* out = a + b (fp16, same shape, n elements, multiple of 8). */
int c2d_add(const void* a, const void* b, void* out, size_t n, void* stream);

/* thread-local hipError_t of the last failed launch (0 if none) */
int c2d_last_hip_error(void);
/* build identification string (arch + git-free version tag) */
const char* c2d_version(void);

#ifdef __cplusplus
}
#endif
#endif /* C2D_H */
