"""SD1.5 UNet2DConditionModel on the HIP kernels (NHWC fp16 activations).

The module tree and attribute names follow diffusers 0.23.1 so that
  - diffusers / SD1.5 checkpoint keys load 1:1 (load_diffusers_state_dict),
  - processor names match ("down_blocks.0.attentions.0.transformer_blocks.0.attn2.processor"),
    which is what the reference AudioProcessorManager keys on
    (models/audio_attention_processor.py:168-193),
  - unet.attn_processors / unet.set_attn_processor behave as in diffusers.

Per-step structure: conv_in, 4 down blocks, mid block, 4 up
blocks, GN+SiLU+conv_out.  Fusions on the HIP path:
  ResnetBlock2D   GN1 stats + apply(SiLU) over the (two-source) skip concat ->
                  conv1 (bias + temb epilogue) -> GN2 stats + apply(SiLU) ->
                  conv2 (bias + residual epilogue); the 1x1 shortcut reads the raw
                  skip concat from its two sources (never materialised);
                  all 22 time_emb_proj GEMMs batched into one (SiLU prologue).
  Transformer2D   GN stats + apply -> proj_in -> block -> proj_out (+residual).
  Block           LN1 -> fused QKV GEMM -> flash attn -> to_out (+residual);
                  LN2 -> audio cross-attn processor (+residual);
                  LN3 -> GEGLU GEMM (h*gelu(g) epilogue) -> Linear (+residual).
  LayerNorm fold  LN1 / LN2 / LN3 run inside the QKV / to_q / GEGLU GEMM where that GEMM is the
                  panel kernel (K = 320 from 8192 rows, K = 640 on its planned shapes): the
                  workgroup normalises its LDS-resident A panel in place and multiplies by
                  W diag(gamma) with bias b + W beta (C2D_PRO_LNFOLD; BasicTransformerBlock._lnf_on;
                  C2D_LN_FOLD=0 materialises the LayerNorm outputs).
  FF out fold     ff.net.2 and proj_out are two linear maps with only a residual add
                  between them: proj_out(h + W2 g + b2) + x = [Wp | Wp W2] [h; g] +
                  (Wp b2 + bp) + x, one K = 5C GEMM reading h and g from their own
                  buffers (Transformer2DModel.finalize / forward; C2D_FOLD_FF_OUT=0
                  keeps the two GEMMs).
  Other normalised activations (GroupNorm) are materialised once per norm (HBM-bound kernels):
  re-normalising inside the consumer GEMM would redo the affine+SiLU in all 9
  taps of a 3x3 conv / every N-tile of a GEMM, which is VALU-bound on CDNA4 -- the panel GEMM
  escapes that because it normalises each A row once, in LDS, for all of its output columns.
  Up/Downsample   stride 2 folded into the conv addressing; the nearest x2 upsample
                  materialised by c2d_upsample_nearest2x (one HBM pass) so the 3x3 conv
                  stays on the LDS-DMA path (Upsample2D below).
  CFG pair        conv_in, the first resnet and the first transformer up to its
                  cross-attention run once per latent (cfg_pair=True); each producer
                  writes the first half of a 2N buffer and one device copy fills the
                  second (forward_nhwc, Transformer2DModel.forward).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import ops
from .layers import HConv2d, HGroupNorm, HLayerNorm, HLinear
from .processor import AttnProcessor, AudioAttnProcessor
from .weights import SD15_UNET

# ff.net.2 folded into proj_out (Transformer2DModel): read once at import, A/B switch only
FOLD_FF_OUT = os.environ.get("C2D_FOLD_FF_OUT", "1") != "0"
# norm1 / norm3 folded into the QKV / GEGLU GEMMs where those run on the panel GEMM (K = 320):
# A/B switch only (C2D_LN_FOLD=0 materialises the LayerNorm outputs)
FOLD_LN = os.environ.get("C2D_LN_FOLD", "1") != "0"
FOLD_LN640 = os.environ.get("C2D_LN_FOLD640", "1") != "0"   # the K = 640 one-round shapes too (round 6; A/B)
# GroupNorm moments from the producing conv (round 6, c2d_conv_desc::gn_mom): norm2 of every ResnetBlock2D and
# the norm after a resnet read the statistics its row-ring conv emitted (one GroupNorm launch instead of two);
# C2D_GN_MOMENTS=0 (A/B) keeps the statistics pass
GN_MOMENTS = os.environ.get("C2D_GN_MOMENTS", "1") != "0"
GN_GROUPS = 32   # every GroupNorm the moments feed (SD1.5 norm_num_groups)
# the CFG-shared prefix (conv_in, the first resnet and self-attention once per latent) from this many latents
# per call: A/B switch (at one latent every kernel is latency bound and the half-batch saves less than the
# duplicating copies cost)
CFG_PREFIX_MIN = int(os.environ.get("C2D_CFG_PREFIX_MIN", "1"))


class Attention(nn.Module):
    """The diffusers Attention surface a processor relies on (to_q/to_k/to_v/
    to_out, heads, scale, spatial_norm, norm_cross, residual_connection,
    rescale_output_factor, head_to_batch_dim, batch_to_head_dim,
    get_attention_scores), plus packed fused weights for the HIP processors."""

    def __init__(self, query_dim: int, cross_attention_dim: int | None = None, heads: int = 8,
                 dim_head: int | None = None, out_bias: bool = True):
        super().__init__()
        dim_head = dim_head or query_dim // heads
        inner = heads * dim_head
        ctx = cross_attention_dim or query_dim
        self.heads, self.dim_head = heads, dim_head
        self.scale = dim_head ** -0.5
        self.is_cross_attention = cross_attention_dim is not None
        self.to_q = HLinear(query_dim, inner, bias=False)
        self.to_k = HLinear(ctx, inner, bias=False)
        self.to_v = HLinear(ctx, inner, bias=False)
        self.to_out = nn.ModuleList([HLinear(inner, query_dim, bias=out_bias), nn.Dropout(0.0)])
        self.spatial_norm = None
        self.norm_cross = None
        self.residual_connection = False
        self.rescale_output_factor = 1.0
        self.upcast_attention = False
        self.upcast_softmax = False
        self.kpad_q = self.to_q.kpad
        self.kpad_kv = self.to_k.kpad
        self.register_buffer("w_qkv", None if self.is_cross_attention else
                             torch.zeros(3 * inner, self.kpad_q, dtype=torch.float16), persistent=False)
        self.register_buffer("w_kv", torch.zeros(2 * inner, self.kpad_kv, dtype=torch.float16), persistent=False)
        self.processor = AttnProcessor()

    @torch.no_grad()
    def finalize(self):
        """Concatenate the packed projections (fused QKV for self-attention, KV for both)."""
        self.w_kv.copy_(torch.cat([self.to_k.weight, self.to_v.weight], 0))
        if self.w_qkv is not None:
            self.w_qkv.copy_(torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight], 0))

    def set_processor(self, processor) -> None:
        self.processor = processor

    def forward(self, hidden_states, encoder_hidden_states=None, attention_mask=None, **cross_attention_kwargs):
        return self.processor(self, hidden_states, encoder_hidden_states=encoder_hidden_states,
                              attention_mask=attention_mask, **cross_attention_kwargs)

    # -- diffusers helpers used by reference-style (torch) processors ----------
    def head_to_batch_dim(self, tensor: torch.Tensor, out_dim: int = 3) -> torch.Tensor:
        b, l, dim = tensor.shape
        h = self.heads
        t = tensor.reshape(b, l, h, dim // h).permute(0, 2, 1, 3)
        return t.reshape(b * h, l, dim // h) if out_dim == 3 else t

    def batch_to_head_dim(self, tensor: torch.Tensor) -> torch.Tensor:
        bh, l, d = tensor.shape
        h = self.heads
        return tensor.reshape(bh // h, h, l, d).permute(0, 2, 1, 3).reshape(bh // h, l, d * h)

    def get_attention_scores(self, query, key, attention_mask=None):
        scores = torch.baddbmm(torch.empty(query.shape[0], query.shape[1], key.shape[1], dtype=query.dtype,
                                           device=query.device), query, key.transpose(-1, -2), beta=0,
                               alpha=self.scale)
        if attention_mask is not None:
            scores = scores + attention_mask
        return scores.softmax(dim=-1).to(query.dtype)


class FeedForward(nn.Module):
    """GEGLU(dim, 4 dim) -> Dropout -> Linear(4 dim, dim); net.0.proj rows packed
    in h/g-interleaved 16-row blocks for the GEGLU epilogue."""

    def __init__(self, dim: int, mult: int = 4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([nn.Module(), nn.Dropout(0.0), HLinear(inner, dim)])
        self.net[0].proj = HLinear(dim, 2 * inner)

    @torch.no_grad()
    def load_geglu(self, w, b):
        wi, bi = ops.geglu_interleave(w.float(), b.float())
        self.net[0].proj.load(wi, bi)


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim: int, heads: int, cross_dim: int):
        super().__init__()
        self.norm1 = HLayerNorm(dim)
        self.attn1 = Attention(dim, None, heads)
        self.norm2 = HLayerNorm(dim)
        self.attn2 = Attention(dim, cross_dim, heads)
        self.norm3 = HLayerNorm(dim)
        self.ff = FeedForward(dim)
        # LayerNorm folded into the GEMM after it (C2D_PRO_LNFOLD, the panel GEMM's K = 320 / 640: the
        # kernel normalises its LDS panel in place): W diag(gamma) and b + W beta for norm1 -> fused
        # QKV, norm2 -> to_q and norm3 -> GEGLU, built by finalize (only with FOLD_LN, so a C2D_LN_FOLD=0
        # model holds no second copy); used where _lnf_on says so, and only once finalize has run
        self.lnf = dim in (320, 640)
        self.lnf_folded = False
        for name in ("qkv", "q", "ff"):
            self.register_buffer(f"lnf_{name}_w", None, persistent=False)
            self.register_buffer(f"lnf_{name}_b", None, persistent=False)

    @torch.no_grad()
    def finalize(self) -> None:
        if not (self.lnf and FOLD_LN):
            return
        c = self.norm1.c
        wq = torch.cat([self.attn1.to_q.weight, self.attn1.to_k.weight, self.attn1.to_v.weight], 0)
        for name, w, b, norm in (("qkv", wq, None, self.norm1), ("q", self.attn2.to_q.weight, None, self.norm2),
                                 ("ff", self.ff.net[0].proj.weight, self.ff.net[0].proj.bias, self.norm3)):
            wf, bf = ops.fold_layernorm(w, b, norm.weight, norm.bias, c)
            setattr(self, f"lnf_{name}_w", wf.contiguous())
            setattr(self, f"lnf_{name}_b", bf.contiguous())
        self.lnf_folded = True

    def _lnf_on(self, m: int, cout: int, geglu: bool) -> bool:
        """Fold the LayerNorm into this GEMM: where the planner runs it on the panel kernel anyway,
        and at K = 320 from 8192 rows on, where the folded panel GEMM beats LayerNorm + the
        planner's tile on every UNet shape measured (profiles/r05_ln_fold.txt: to_q 320 -> 320 at
        c3 42.8 -> 34.7 us, c5's fused QKV 105.9 -> 92.4); at K = 640 (one 160-KiB panel workgroup
        per CU) from 8192 rows where the panels x column splits fit one round of 256 CUs (c3 level 1:
        QKV 66.7 -> 65.8, to_q 34.4 -> 32.3 us before the LayerNorm launch's in-situ gap; c5's
        18432 rows take 288 workgroups and lose: 76.2 -> 115.3)."""
        c = self.norm1.c
        if not (self.lnf_folded and ops.panel_gemm(m, c, cout, geglu, lnfold=True)):
            return False
        if ops.panel_gemm(m, c, cout, geglu) or (c == 320 and m >= 8192):
            return True
        if c == 640 and m >= 8192 and FOLD_LN640:
            panels = (m + 127) // 128
            ns = min(max((256 + panels - 1) // panels, 1), ((cout >> 5) + 7) // 8)   # igemm_panel.h panel_nsplit
            return panels * ns <= 256
        return False

    def _attend(self, attn: Attention, x, h, ehs, mask, kwargs):
        if getattr(attn.processor, "fuses_residual", False):
            return attn(x, encoder_hidden_states=ehs, attention_mask=mask, _residual=h, **kwargs)
        # a diffusers-style processor (torch ops, e.g. the reference's own): its output
        # plus the block residual, as BasicTransformerBlock adds it
        out = attn(x, encoder_hidden_states=ehs, attention_mask=mask, **kwargs)
        return ops.add(out.to(h.dtype).contiguous(), h)

    def forward(self, h: torch.Tensor, ehs: torch.Tensor, cross_attention_kwargs: dict,
                encoder_attention_mask: torch.Tensor | None = None,
                cfg_dup: torch.Tensor | None = None) -> torch.Tensor:
        """The whole block: attention part (forward_attn) -> LN3 -> GEGLU -> Linear
        (+residual, in place in h)."""
        h = self.forward_attn(h, ehs, cross_attention_kwargs, encoder_attention_mask, cfg_dup)
        b, l, c = h.shape
        h2 = h.view(b * l, c)
        self.ff.net[2](self.ff_inner(h2), resid=h2, out=h2)
        return h

    def ff_inner(self, h2: torch.Tensor) -> torch.Tensor:
        """GEGLU(LN3(h)) [M, 4C]: the feed-forward up to its output Linear (LN3 folded into the
        GEMM on panel-GEMM shapes)."""
        proj = self.ff.net[0].proj
        if self._lnf_on(h2.shape[0], proj.out_features, True):
            return ops.conv(h2, self.lnf_ff_w, proj.kpad, proj.out_features, ksize=1, bias=self.lnf_ff_b,
                            act="geglu", ln_fold=self.norm3.eps)
        return proj(self.norm3(h2), act="geglu")

    def forward_attn(self, h: torch.Tensor, ehs: torch.Tensor, cross_attention_kwargs: dict,
                     encoder_attention_mask: torch.Tensor | None = None,
                     cfg_dup: torch.Tensor | None = None) -> torch.Tensor:
        """h: [B, L, C] fp16 (updated in place by the fused residual epilogues).
        encoder_attention_mask: additive key bias for attn2 (diffusers BasicTransformerBlock).
        cfg_dup: h holds one half of a CFG pair whose halves are identical up to here, and is the
        first half of this [2B, L, C] buffer; the self-attention runs on it once and its output
        is copied into the second half before attn2, the first op where the [uncond, cond] halves
        differ (UNet2DConditionModel.forward_nhwc)."""
        kw = cross_attention_kwargs or {}
        b, l, c = h.shape
        inner = self.attn1.heads * self.attn1.dim_head
        if type(self.attn1.processor) is AttnProcessor and self._lnf_on(b * l, 3 * inner, False):
            # norm1 folded into the fused QKV GEMM; the stock processor takes the projections
            qkv = ops.conv(h.view(b * l, c), self.lnf_qkv_w, self.attn1.kpad_q, 3 * inner, ksize=1,
                           bias=self.lnf_qkv_b, ln_fold=self.norm1.eps)
            h = self._attend(self.attn1, h, h, None, None, dict(kw, _qkv=qkv))
        else:
            h = self._attend(self.attn1, self.norm1(h), h, None, None, kw)
        if cfg_dup is not None:
            n = h.shape[0]
            if h.data_ptr() != cfg_dup.data_ptr():   # a plugin processor returned a new tensor
                cfg_dup[:n].copy_(h)
            cfg_dup[n:].copy_(cfg_dup[:n])
            h = cfg_dup
        b, l, c = h.shape
        if type(self.attn2.processor) in (AttnProcessor, AudioAttnProcessor) and self._lnf_on(b * l, inner, False):
            # norm2 folded into to_q; the stock / audio processor takes the projected query
            q = ops.conv(h.view(b * l, c), self.lnf_q_w, self.attn2.kpad_q, inner, ksize=1, bias=self.lnf_q_b,
                         ln_fold=self.norm2.eps)
            return self._attend(self.attn2, h, h, ehs, encoder_attention_mask, dict(kw, _q=q))
        return self._attend(self.attn2, self.norm2(h), h, ehs, encoder_attention_mask, kw)


class Transformer2DModel(nn.Module):
    def __init__(self, c: int, heads: int, cross_dim: int, groups: int = 32):
        super().__init__()
        self.norm = HGroupNorm(groups, c, 1e-6)
        self.proj_in = HConv2d(c, c, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(c, heads, cross_dim)])
        self.proj_out = HConv2d(c, c, 1)
        # [Wp | Wp W2] packed for the K = 5C GEMM over [h; GEGLU(LN3(h))] (finalize)
        # (the two-source GEMM reads h as whole 64-channel K steps: C % 64 == 0, as in SD1.5)
        self.fold_kpad = ops.kpad_of(5 * c)
        self.fold_ok = c % 64 == 0
        self.register_buffer("w_out_fold", torch.zeros(c, self.fold_kpad, dtype=torch.float16), persistent=False)
        self.register_buffer("b_out_fold", torch.zeros(c, dtype=torch.float32), persistent=False)

    @torch.no_grad()
    def finalize(self) -> None:
        """Fold the feed-forward's output Linear into proj_out (both 1x1 maps on the C
        channels, only the block residual between them): Wf = Wp W2 in fp32 from the fp16
        weights, rounded once; bias Wp b2 + bp.  Also finalizes the block (its LayerNorm folds), so a
        standalone Transformer2DModel is complete after this call."""
        for blk in self.transformer_blocks:
            blk.finalize()
        if not self.fold_ok:
            return
        c = self.proj_out.cout
        wp = self.proj_out.weight[:, :c].float()
        ff2 = self.transformer_blocks[0].ff.net[2]
        w2 = ff2.weight[:, :4 * c].float()
        self.w_out_fold.copy_(torch.cat([wp, wp @ w2], 1).to(torch.float16))
        self.b_out_fold.copy_(wp @ ff2.bias.float() + self.proj_out.bias.float())

    def _block_out(self, t: torch.Tensor, x4: torch.Tensor, resid: torch.Tensor, gm: int = 0):
        """Feed-forward + proj_out (+ resid) of the attention-part output t [B, L, C]:
        proj_out(t + ff(t)) + resid, as one K = 5C GEMM over [t; GEGLU(LN3(t))].  gm > 0: (out, the
        GroupNorm moments over gm groups the GEMM emitted for the next norm, or None)."""
        blk = self.transformer_blocks[0]
        b, l, c = t.shape
        hh, ww = x4.shape[1], x4.shape[2]
        t2 = t.view(b * l, c)
        ff1 = blk.ff_inner(t2)
        r = ops.conv(t2.view(b, hh, ww, c), self.w_out_fold, self.fold_kpad, c, ksize=1, bias=self.b_out_fold,
                     x2=ff1.view(b, hh, ww, ff1.shape[-1]), resid=resid.reshape(b, hh, ww, c),
                     gn_moments=gm)
        return r

    def forward(self, x, ehs, cross_attention_kwargs, encoder_attention_mask=None,
                cfg_dup: torch.Tensor | None = None, x_mom=None, want_mom: bool = False):
        """cfg_dup: x is one half of a CFG pair with identical halves and the first half of this
        [2N, H, W, C] buffer; the output is the full pair (the block duplicates its state before
        the cross-attention, and x into the buffer's second half for proj_out's residual).  The
        duplicates are one device copy of a half each -- a torch.cat of the halves read 1 and
        wrote 2 half-tensors (30 us per call at level 0).  x_mom: x's GroupNorm moments from its
        producer (ops.GnMoments) for self.norm; want_mom: return (out, the moments of out that its
        GEMM emitted for the next norm, or None)."""
        gm = GN_GROUPS if want_mom and GN_MOMENTS else 0
        r = self._forward(x, ehs, cross_attention_kwargs, encoder_attention_mask, cfg_dup, x_mom, gm)
        if want_mom and not gm:
            return r, None
        return r

    def _forward(self, x, ehs, cross_attention_kwargs, encoder_attention_mask, cfg_dup, x_mom, gm):
        n, hh, ww, c = x.shape
        blk = self.transformer_blocks[0]
        fold = FOLD_FF_OUT and self.fold_ok
        if cfg_dup is None:
            h = self.proj_in(self.norm.apply(x, mom=x_mom))
            if fold:
                t = blk.forward_attn(h.view(n, hh * ww, c), ehs, cross_attention_kwargs, encoder_attention_mask)
                return self._block_out(t, x, x, gm)
            t = blk(h.view(n, hh * ww, c), ehs, cross_attention_kwargs, encoder_attention_mask)
            return self.proj_out(t.view(n, hh, ww, c), resid=x, gn_moments=gm)
        hb = x.new_empty((2 * n, hh * ww, c))
        h = self.proj_in(self.norm.apply(x, mom=x_mom), out=hb[:n].view(n, hh, ww, c))
        if fold:
            t = blk.forward_attn(h.view(n, hh * ww, c), ehs, cross_attention_kwargs, encoder_attention_mask,
                                 cfg_dup=hb)
            cfg_dup[n:].copy_(cfg_dup[:n])
            return self._block_out(t, cfg_dup, cfg_dup, gm)
        t = blk(h.view(n, hh * ww, c), ehs, cross_attention_kwargs, encoder_attention_mask, cfg_dup=hb)
        cfg_dup[n:].copy_(cfg_dup[:n])
        return self.proj_out(t.view(2 * n, hh, ww, c), resid=cfg_dup, gn_moments=gm)


class ResnetBlock2D(nn.Module):
    def __init__(self, cin: int, cout: int, temb_ch: int = 1280, groups: int = 32, eps: float = 1e-5):
        super().__init__()
        self.cin, self.cout = cin, cout
        self.norm1 = HGroupNorm(groups, cin, eps)
        self.conv1 = HConv2d(cin, cout, 3)
        self.time_emb_proj = HLinear(temb_ch, cout) if temb_ch else None
        self.norm2 = HGroupNorm(groups, cout, eps)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = HConv2d(cout, cout, 3)
        self.conv_shortcut = HConv2d(cin, cout, 1) if cin != cout else None
        self.temb_off = None  # column offset into the batched time_emb_proj output

    def forward(self, x, temb_all=None, skip=None, out=None, x_mom=None, want_mom: bool = False):
        """x_mom: x's GroupNorm moments from its producer (ops.GnMoments) for norm1; want_mom: return
        (out, moments of out for a following 32-group norm, or None).  conv1 emits norm2's moments
        itself where the library can (the row-ring tiles: c2d_conv2d_gn_rows), so norm2 is one launch."""
        temb = None
        if temb_all is not None:
            temb = temb_all[:, self.temb_off:self.temb_off + self.cout]
        n, hh, ww, _ = x.shape
        cin = self.cin
        # act(GroupNorm) in the zero-bordered layout where the conv planner runs the row-ring 3x3
        # (tile 42: the c3 batch's level-0 convs), the plain layout elsewhere
        p1 = ops.rowring_conv(n, hh, ww, cin, self.cout)
        a1 = self.norm1.apply(x, skip, silu=True, pad=p1, mom=x_mom if skip is None else None)
        if GN_MOMENTS:
            h, hm = self.conv1(a1, temb=temb, padded=p1, gn_moments=self.norm2.num_groups)
        else:
            h, hm = self.conv1(a1, temb=temb, padded=p1), None
        res = self.conv_shortcut(x, x2=skip) if self.conv_shortcut is not None else x
        p2 = ops.rowring_conv(n, hh, ww, self.cout, self.cout)
        y = self.conv2(self.norm2.apply(h, silu=True, pad=p2, mom=hm), resid=res, out=out, padded=p2,
                       gn_moments=self.norm2.num_groups if want_mom and GN_MOMENTS else 0)
        return (y, None) if want_mom and not GN_MOMENTS else y


class Downsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = HConv2d(c, c, 3, stride=2)

    def forward(self, x, want_mom: bool = False):
        """want_mom: (out, its GroupNorm moments for the next resnet's norm1, or None)."""
        if want_mom and GN_MOMENTS:
            return self.conv(x, gn_moments=GN_GROUPS)
        return (self.conv(x), None) if want_mom else self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = HConv2d(c, c, 3)

    def forward(self, x):
        # materialised x2 (one HBM pass) keeps the conv on the LDS-DMA path
        return self.conv(ops.upsample_nearest2x(x))


class _Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.resnets = nn.ModuleList()
        self.attentions = nn.ModuleList()


class TimestepEmbedding(nn.Module):
    def __init__(self, cin: int, dim: int):
        super().__init__()
        self.linear_1 = HLinear(cin, dim)
        self.linear_2 = HLinear(dim, dim)

    def forward(self, t_sin):
        return self.linear_2(self.linear_1(t_sin, act="silu"))


class UNetOutput:
    def __init__(self, sample):
        self.sample = sample

    def __getitem__(self, i):
        return (self.sample,)[i]


class UNet2DConditionModel(nn.Module):
    def __init__(self, cfg: dict = SD15_UNET):
        super().__init__()
        self.cfg = dict(cfg)
        ch = cfg["block_out_channels"]
        heads, ctx, groups = cfg["heads"], cfg["cross_attention_dim"], cfg["norm_groups"]
        temb_ch = ch[0] * 4
        self.in_pad = 8
        self.conv_in = HConv2d(cfg["in_channels"], ch[0], 3, cin_pad=self.in_pad)
        self.time_embedding = TimestepEmbedding(ch[0], temb_ch)
        self.down_blocks = nn.ModuleList()
        out_c = ch[0]
        for i, c in enumerate(ch):
            blk = _Block()
            in_c, out_c = out_c, c
            for j in range(cfg["layers_per_block"]):
                blk.resnets.append(ResnetBlock2D(in_c if j == 0 else out_c, out_c, temb_ch, groups))
                if cfg["attn_blocks"][i]:
                    blk.attentions.append(Transformer2DModel(out_c, heads, ctx, groups))
            if i < len(ch) - 1:
                blk.downsamplers = nn.ModuleList([Downsample2D(out_c)])
            self.down_blocks.append(blk)
        self.mid_block = _Block()
        self.mid_block.resnets.append(ResnetBlock2D(ch[-1], ch[-1], temb_ch, groups))
        self.mid_block.attentions.append(Transformer2DModel(ch[-1], heads, ctx, groups))
        self.mid_block.resnets.append(ResnetBlock2D(ch[-1], ch[-1], temb_ch, groups))
        self.up_blocks = nn.ModuleList()
        rev = list(reversed(ch))
        rev_attn = list(reversed(cfg["attn_blocks"]))
        out_c = rev[0]
        n_up = cfg["layers_per_block"] + 1
        for i in range(len(rev)):
            blk = _Block()
            prev_c, out_c = out_c, rev[i]
            in_c = rev[min(i + 1, len(rev) - 1)]
            for j in range(n_up):
                skip = in_c if j == n_up - 1 else out_c
                r_in = prev_c if j == 0 else out_c
                blk.resnets.append(ResnetBlock2D(r_in + skip, out_c, temb_ch, groups))
                blk.resnets[-1].skip_ch = skip
                if rev_attn[i]:
                    blk.attentions.append(Transformer2DModel(out_c, heads, ctx, groups))
            if i < len(rev) - 1:
                blk.upsamplers = nn.ModuleList([Upsample2D(out_c)])
            self.up_blocks.append(blk)
        self.conv_norm_out = HGroupNorm(groups, ch[0], cfg["norm_eps"])
        self.conv_out = HConv2d(ch[0], cfg["out_channels"], 3)
        resnets = [m for m in self.modules() if isinstance(m, ResnetBlock2D)]
        off = 0
        for r in resnets:
            r.temb_off = off
            off += r.cout
        self.temb_total = off
        kp = ops.kpad_of(temb_ch)
        self.register_buffer("w_temb_all", torch.zeros(off, kp, dtype=torch.float16), persistent=False)
        self.register_buffer("b_temb_all", torch.zeros(off, dtype=torch.float32), persistent=False)
        self.temb_kpad = kp

    # ------------------------------------------------------------ weights
    @torch.no_grad()
    def load_diffusers_state_dict(self, sd: dict) -> None:
        """Load diffusers-0.23.1 UNet2DConditionModel keys (SD1.5 layout)."""
        used = set()
        for name, m in self.named_modules():
            if isinstance(m, FeedForward):
                k = name + ".net.0.proj"
                m.load_geglu(sd[k + ".weight"], sd[k + ".bias"])
                used |= {k + ".weight", k + ".bias"}
        for name, m in self.named_modules():
            if isinstance(m, (HLinear, HConv2d, HGroupNorm, HLayerNorm)):
                if name.endswith("net.0.proj"):
                    continue
                wk, bk = name + ".weight", name + ".bias"
                m.load(sd[wk], sd.get(bk))
                used |= {wk, bk}
        missing = [k for k in sd if k not in used]
        if missing:
            raise KeyError(f"unused checkpoint keys: {missing[:5]} ...")
        self.finalize()

    @torch.no_grad()
    def finalize(self) -> None:
        for m in self.modules():
            if isinstance(m, (Attention, Transformer2DModel)):   # Transformer2DModel finalizes its blocks
                m.finalize()
        rs = [m for m in self.modules() if isinstance(m, ResnetBlock2D)]
        self.w_temb_all.copy_(torch.cat([r.time_emb_proj.weight for r in rs], 0))
        self.b_temb_all.copy_(torch.cat([r.time_emb_proj.bias for r in rs], 0))

    # ------------------------------------------------------------ processors
    @property
    def attn_processors(self) -> dict:
        return {f"{n}.processor": m.processor for n, m in self.named_modules() if isinstance(m, Attention)}

    def set_attn_processor(self, processor) -> None:
        for n, m in self.named_modules():
            if isinstance(m, Attention):
                m.set_processor(processor[f"{n}.processor"] if isinstance(processor, dict) else processor)

    # ------------------------------------------------------------ forward
    def time_conditioning(self, t_sin: torch.Tensor) -> torch.Tensor:
        """t_sin [M, 320] fp16 sinusoidal embedding -> every resnet's time_emb_proj(silu(
        TimestepEmbedding(t))) side by side, [M, 22 x cout] fp16 (resnet r at temb_off)."""
        temb = self.time_embedding(t_sin)
        return ops.conv(temb, self.w_temb_all, self.temb_kpad, self.temb_total, ksize=1, bias=self.b_temb_all,
                        silu_in=True)

    def cfg_shared_prefix_ok(self) -> bool:
        """The [uncond, cond] halves of a CFG batch see the same latent, timestep and (per the
        composition contract) audio tokens; they first differ at the first cross-attention,
        where the text context enters (down_blocks.0.attentions.0...attn2).  Everything before
        it -- conv_in, the first ResnetBlock2D, that transformer's GroupNorm, proj_in, LayerNorm
        and self-attention -- can run on one half and be duplicated, when the self-attention
        there runs the stock processor (a plugin on attn1 may use per-half kwargs)."""
        blk = self.down_blocks[0]
        if not len(blk.attentions):
            return False
        return type(blk.attentions[0].transformer_blocks[0].attn1.processor) is AttnProcessor

    def forward_nhwc(self, x: torch.Tensor, t_sin: torch.Tensor | None, ehs: torch.Tensor,
                     cross_attention_kwargs: dict | None = None,
                     encoder_attention_mask: torch.Tensor | None = None,
                     temb_all: torch.Tensor | None = None, cfg_pair: bool = False) -> torch.Tensor:
        """x: [N, H, W, 8] fp16 (latent zero-padded to 8 ch); t_sin: [N, 320] fp16
        sinusoidal embedding; ehs: [N, 77, 768] fp16; encoder_attention_mask: additive
        key bias [N, 1, 77] for every attn2 (or None); temb_all: precomputed
        time_conditioning rows [N, 22 x cout] (any row stride, 0 = one row for all) in place
        of t_sin.  cfg_pair: x holds N/2 latents and the UNet batch is the CFG pair [x; x]
        (the prefix before the first cross-attention then runs once per latent,
        cfg_shared_prefix_ok); t_sin / temb_all rows must then be the same for both halves.
        Returns eps [N, H, W, 4] fp16."""
        kw = cross_attention_kwargs or {}
        em = encoder_attention_mask
        if temb_all is None:
            temb_all = self.time_conditioning(t_sin)
        shared = cfg_pair and x.shape[0] >= CFG_PREFIX_MIN and self.cfg_shared_prefix_ok()
        if cfg_pair and not shared:
            x = torch.cat([x, x], 0)
        if shared:   # conv_in runs on one half, written into the first half of the skip buffer
            n0 = x.shape[0]
            skip0 = x.new_empty((2 * n0, x.shape[1], x.shape[2], self.conv_in.cout))
            h = self.conv_in(x, out=skip0[:n0])
            skip0[n0:].copy_(skip0[:n0])
            skips = [skip0]
        else:
            h = self.conv_in(x)
            skips = [h]
        # hm: GroupNorm moments of h from the conv that produced it (ops.GnMoments, or None), for the
        # next norm over h (a transformer's norm, the next resnet's norm1); anything else drops them
        hm = None
        for i, blk in enumerate(self.down_blocks):
            for j, r in enumerate(blk.resnets):
                pre = shared and i == 0 and j == 0   # still on one half of the CFG pair
                if pre:   # the resnet output lands in the first half of its CFG-pair buffer
                    hb = h.new_empty((2 * h.shape[0], h.shape[1], h.shape[2], r.cout))
                    h, hm = r(h, temb_all, out=hb[:h.shape[0]], x_mom=hm, want_mom=True)
                else:
                    h, hm = r(h, temb_all, x_mom=hm, want_mom=True)
                if len(blk.attentions):
                    h, hm = blk.attentions[j](h, ehs, kw, em, cfg_dup=hb if pre else None, x_mom=hm, want_mom=True)
                elif pre:
                    hb[h.shape[0]:].copy_(h)
                    h, hm = hb, None
                skips.append(h)
            if hasattr(blk, "downsamplers"):
                h, hm = blk.downsamplers[0](h, want_mom=True)
                skips.append(h)
        mb = self.mid_block
        h, hm = mb.resnets[0](h, temb_all, x_mom=hm, want_mom=True)
        h, hm = mb.attentions[0](h, ehs, kw, em, x_mom=hm, want_mom=True)
        h = mb.resnets[1](h, temb_all, x_mom=hm)
        for blk in self.up_blocks:
            for j, r in enumerate(blk.resnets):   # norm1 over [h; skip]: no producer moments
                h, hm = r(h, temb_all, skip=skips.pop(), want_mom=True)
                if len(blk.attentions):
                    h, hm = blk.attentions[j](h, ehs, kw, em, x_mom=hm, want_mom=True)
                else:
                    hm = None
            if hasattr(blk, "upsamplers"):
                h, hm = blk.upsamplers[0](h), None
        return self.conv_out(self.conv_norm_out.apply(h, silu=True, mom=hm))

    def forward(self, sample: torch.Tensor, timestep, encoder_hidden_states: torch.Tensor,
                cross_attention_kwargs: dict | None = None, return_dict: bool = True,
                encoder_attention_mask: torch.Tensor | None = None):
        """diffusers-compatible entry: sample [N, 4, H, W] -> eps [N, 4, H, W] fp16.
        encoder_attention_mask [N, 77] (1 = keep, 0 = discard) becomes the additive bias
        (1 - mask) * -10000 of every cross-attention, as diffusers 0.23.1 builds it."""
        n = sample.shape[0]
        x = ops.latent_to_nhwc(sample.float().contiguous(), self.in_pad, dup=False)
        t = torch.as_tensor(timestep, dtype=torch.float32, device=sample.device).reshape(-1)
        if t.numel() == 1:
            t_sin = ops.timestep_embedding(t.contiguous(), None, n, self.cfg["block_out_channels"][0])
        else:  # per-sample timesteps: one row at a time through the same kernel
            t_sin = torch.cat([ops.timestep_embedding(t[i:i + 1].contiguous(), None, 1,
                                                      self.cfg["block_out_channels"][0]) for i in range(n)])
        ehs = encoder_hidden_states.to(torch.float16).contiguous()
        em = None
        if encoder_attention_mask is not None:
            em = ((1.0 - encoder_attention_mask.float()) * -10000.0).unsqueeze(1)
        eps = self.forward_nhwc(x, t_sin, ehs, cross_attention_kwargs, em)
        out = eps.permute(0, 3, 1, 2).contiguous()
        return UNetOutput(out) if return_dict else (out,)
