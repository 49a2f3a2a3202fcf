"""fp32 CPU restatement of the SD1.5 AutoencoderKL decoder (TEST ORACLE ONLY).

diffusers==0.23.1 semantics (absent here; parity unpinned by the reference):
post_quant_conv 1x1, Decoder(conv_in, UNetMidBlock2D(resnet, Attention(1 head,
GN eps 1e-6, residual), resnet), 4 UpDecoderBlock2D of 3 resnets (eps 1e-6)
+ nearest-x2 upsample conv, GN+SiLU, conv_out); image = (x/2 + 0.5).clamp(0, 1);
latents are divided by the 0.18215 scaling factor first.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class VAEDecoderRef:
    def __init__(self, sd: dict, groups: int = 32):
        self.sd = {k: v.float() for k, v in sd.items()}
        self.g = groups

    def conv(self, k, x):
        w = self.sd[k + ".weight"]
        return F.conv2d(x, w, self.sd[k + ".bias"], padding=w.shape[-1] // 2)

    def gn(self, k, x):
        return F.group_norm(x, self.g, self.sd[k + ".weight"], self.sd[k + ".bias"], 1e-6)

    def resnet(self, k, x):
        h = self.conv(k + ".conv1", F.silu(self.gn(k + ".norm1", x)))
        h = self.conv(k + ".conv2", F.silu(self.gn(k + ".norm2", h)))
        if k + ".conv_shortcut.weight" in self.sd:
            x = self.conv(k + ".conv_shortcut", x)
        return x + h

    def attn(self, k, x):
        b, c, h, w = x.shape
        y = self.gn(k + ".group_norm", x).view(b, c, h * w).transpose(1, 2)
        q = F.linear(y, self.sd[k + ".to_q.weight"], self.sd[k + ".to_q.bias"])
        kk = F.linear(y, self.sd[k + ".to_k.weight"], self.sd[k + ".to_k.bias"])
        v = F.linear(y, self.sd[k + ".to_v.weight"], self.sd[k + ".to_v.bias"])
        p = torch.softmax(q @ kk.transpose(1, 2) / c ** 0.5, dim=-1)
        o = F.linear(p @ v, self.sd[k + ".to_out.0.weight"], self.sd[k + ".to_out.0.bias"])
        return o.transpose(1, 2).reshape(b, c, h, w) + x

    def __call__(self, latents: torch.Tensor) -> torch.Tensor:
        """-> float image in [0, 1], NCHW."""
        x = self.conv("post_quant_conv", latents.float() / 0.18215)
        x = self.conv("decoder.conv_in", x)
        x = self.resnet("decoder.mid_block.resnets.0", x)
        x = self.attn("decoder.mid_block.attentions.0", x)
        x = self.resnet("decoder.mid_block.resnets.1", x)
        for i in range(4):
            for j in range(3):
                x = self.resnet(f"decoder.up_blocks.{i}.resnets.{j}", x)
            if f"decoder.up_blocks.{i}.upsamplers.0.conv.weight" in self.sd:
                x = self.conv(f"decoder.up_blocks.{i}.upsamplers.0.conv", F.interpolate(x, scale_factor=2.0))
        x = self.conv("decoder.conv_out", F.silu(self.gn("decoder.conv_norm_out", x)))
        return (x / 2 + 0.5).clamp(0, 1)
