"""SD1.5 AutoencoderKL decoder (latent [B,4,h,w] -> image [B,8h,8w,3] uint8).

SURVEY.md §8(f) "next" #1.  Convolutions, GroupNorm(+SiLU) and the resnet /
upsample structure reuse the UNet's HIP kernels (NHWC fp16, implicit GEMM with
fused GN prologue and residual epilogue); the single-head d=512 mid-block
attention runs through torch SDPA on the HIP-produced Q/K/V for now.
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
    def __init__(self, c: int, groups: int = 32):
        super().__init__()
        self.c = c
        self.group_norm = HGroupNorm(groups, c, 1e-6)
        self.to_q, self.to_k, self.to_v = HLinear(c, c), HLinear(c, c), HLinear(c, c)
        self.to_out = nn.ModuleList([HLinear(c, c)])
        self.register_buffer("w_qkv", torch.zeros(3 * c, ops.kpad_of(c), dtype=torch.float16), persistent=False)
        self.register_buffer("b_qkv", torch.zeros(3 * c), persistent=False)

    @torch.no_grad()
    def finalize(self):
        self.w_qkv.copy_(torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight]))
        self.b_qkv.copy_(torch.cat([self.to_q.bias, self.to_k.bias, self.to_v.bias]))

    def forward(self, x):
        b, h, w, c = x.shape
        qkv = ops.conv(self.group_norm.apply(x), self.w_qkv, ops.kpad_of(c), 3 * c, ksize=1, bias=self.b_qkv)
        qkv = qkv.view(b, 1, h * w, 3 * c)
        o = F.scaled_dot_product_attention(qkv[..., :c], qkv[..., c:2 * c], qkv[..., 2 * c:])
        return self.to_out[0](o.reshape(b * h * w, c).contiguous(), resid=x.view(b * h * w, c)).view(b, h, w, c)


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
