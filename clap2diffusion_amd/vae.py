"""SD1.5 AutoencoderKL decoder (latent [B,4,h,w] -> image [B,8h,8w,3] uint8).

SURVEY.md §8(f) "next" #1.  Convolutions, GroupNorm(+SiLU) and the resnet /
upsample structure reuse the UNet's HIP kernels (NHWC fp16, implicit GEMM with
fused GN prologue and residual epilogue); the single-head d=512 mid-block
attention is materialised per image on the same GEMM kernel (S = Q K^T, HIP row
softmax, O = P V) -- a 512-wide head does not fit the flash kernel's registers.
diffusers-0.23.1 AutoencoderKL decoder keys (post_quant_conv.*, decoder.*).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .layers import HConv2d, HGroupNorm, HLinear
from .unet import ResnetBlock2D, Upsample2D
from .weights import SD15_VAE

SCALING = 0.18215


class VAEAttention(nn.Module):
    """diffusers Attention(c, heads=1, dim_head=c) with its GroupNorm, as in the
    AutoencoderKL mid block: x + to_out(softmax(q k^T / sqrt(c)) v)."""

    def __init__(self, c: int, groups: int = 32):
        super().__init__()
        self.c = c
        self.group_norm = HGroupNorm(groups, c, 1e-6)
        self.to_q, self.to_k, self.to_v = HLinear(c, c), HLinear(c, c), HLinear(c, c)
        self.to_out = nn.ModuleList([HLinear(c, c)])
        # to_q with the 1/sqrt(c) score scale folded in (keeps fp16 scores 22x away from overflow)
        self.register_buffer("w_qs", torch.zeros(c, ops.kpad_of(c), dtype=torch.float16), persistent=False)
        self.register_buffer("b_qs", torch.zeros(c), persistent=False)

    @torch.no_grad()
    def finalize(self):
        sc = self.c ** -0.5
        self.w_qs.copy_((self.to_q.weight.float() * sc).half())
        self.b_qs.copy_(self.to_q.bias * sc)

    def forward(self, x):
        b, h, w, c = x.shape
        hw = h * w
        assert hw % 64 == 0 and c % 64 == 0, "VAE attention needs h*w and c multiples of 64"
        xn = self.group_norm.apply(x).view(b * hw, c)
        q = ops.conv(xn, self.w_qs, c, c, ksize=1, bias=self.b_qs)
        k = ops.conv(xn, self.to_k.weight, c, c, ksize=1, bias=self.to_k.bias)
        o = torch.empty_like(q)
        vt = torch.empty(c, hw, device=x.device, dtype=torch.float16)
        s = torch.empty(hw, hw, device=x.device, dtype=torch.float16)
        for i in range(b):
            rows = slice(i * hw, (i + 1) * hw)
            # V^T = W_v X^T: X is the "weight" operand, so the product lands transposed;
            # b_v rides the PV epilogue instead (softmax rows sum to 1)
            ops.conv(self.to_v.weight, xn[rows], c, hw, ksize=1, out=vt)
            ops.conv(q[rows], k[rows], c, hw, ksize=1, out=s)
            ops.softmax_rows(s, out=s)
            ops.conv(s, vt, hw, c, ksize=1, bias=self.to_v.bias, out=o[rows])
        return self.to_out[0](o, resid=x.view(b * hw, c)).view(b, h, w, c)


class VAEDecoder(nn.Module):
    def __init__(self, cfg: dict = SD15_VAE):
        super().__init__()
        ch = list(reversed(cfg["block_out_channels"]))
        g = cfg["norm_groups"]
        self.post_quant_conv = HConv2d(4, 8, 1, cin_pad=8)    # output padded to 8 ch for conv_in
        dec = nn.Module()
        dec.conv_in = HConv2d(4, ch[0], 3, cin_pad=8)
        dec.mid_block = nn.Module()
        dec.mid_block.resnets = nn.ModuleList([ResnetBlock2D(ch[0], ch[0], 0, g, 1e-6),
                                               ResnetBlock2D(ch[0], ch[0], 0, g, 1e-6)])
        dec.mid_block.attentions = nn.ModuleList([VAEAttention(ch[0], g)])
        dec.up_blocks = nn.ModuleList()
        out_c = ch[0]
        for i, c in enumerate(ch):
            blk = nn.Module()
            prev, out_c = out_c, c
            blk.resnets = nn.ModuleList([ResnetBlock2D(prev if j == 0 else out_c, out_c, 0, g, 1e-6)
                                         for j in range(cfg["layers_per_block"] + 1)])
            if i < len(ch) - 1:
                blk.upsamplers = nn.ModuleList([Upsample2D(out_c)])
            dec.up_blocks.append(blk)
        dec.conv_norm_out = HGroupNorm(g, ch[-1], 1e-6)
        dec.conv_out = HConv2d(ch[-1], 4, 3)                   # 3 RGB + 1 zero channel
        self.decoder = dec

    @torch.no_grad()
    def load_diffusers_state_dict(self, sd: dict) -> None:
        used = set()
        pw, pb = sd["post_quant_conv.weight"], sd["post_quant_conv.bias"]
        self.post_quant_conv.load(F.pad(pw, (0, 0, 0, 0, 0, 0, 0, 4)), F.pad(pb, (0, 4)))
        ow, ob = sd["decoder.conv_out.weight"], sd["decoder.conv_out.bias"]
        self.decoder.conv_out.load(F.pad(ow, (0, 0, 0, 0, 0, 0, 0, 1)), F.pad(ob, (0, 1)))
        used |= {"post_quant_conv.weight", "post_quant_conv.bias", "decoder.conv_out.weight", "decoder.conv_out.bias"}
        for name, m in self.decoder.named_modules():
            if isinstance(m, (HLinear, HConv2d, HGroupNorm)) and name != "conv_out":
                k = "decoder." + name
                m.load(sd[k + ".weight"], sd.get(k + ".bias"))
                used |= {k + ".weight", k + ".bias"}
        left = [k for k in sd if k not in used]
        if left:
            raise KeyError(f"unused VAE keys: {left[:4]}")
        self.decoder.mid_block.attentions[0].finalize()

    @torch.no_grad()
    def forward(self, latents: torch.Tensor) -> torch.Tensor:
        """latents [B,4,h,w] fp32 -> uint8 image NHWC [B, 8h, 8w, 3]."""
        d = self.decoder
        z = ops.latent_to_nhwc((latents.float() / SCALING).contiguous(), 8, dup=False)
        x = d.conv_in(self.post_quant_conv(z))
        x = d.mid_block.resnets[0](x)
        x = d.mid_block.attentions[0](x)
        x = d.mid_block.resnets[1](x)
        for blk in d.up_blocks:
            for r in blk.resnets:
                x = r(x)
            if hasattr(blk, "upsamplers"):
                x = blk.upsamplers[0](x)
        x = d.conv_out(d.conv_norm_out.apply(x, silu=True))
        img = (x[..., :3].float() / 2 + 0.5).clamp_(0, 1)
        return (img * 255).round_().to(torch.uint8)
