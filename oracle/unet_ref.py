"""fp32 CPU restatement of the SD1.5 UNet2DConditionModel forward with the
reference AudioAttnProcessor in every cross-attention (TEST ORACLE ONLY).

Third-party semantics restated from diffusers==0.23.1 (requirements.txt:7 of the
reference; not installed anywhere here) per SURVEY.md Appendix A:
  get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0),
  TimestepEmbedding(linear_1, SiLU, linear_2), ResnetBlock2D (GN 32 eps 1e-5,
  SiLU, conv3x3, + time_emb_proj(SiLU(temb)), GN, SiLU, conv3x3, + shortcut),
  Transformer2DModel (GN eps 1e-6, proj_in 1x1 conv, BasicTransformerBlock,
  proj_out, + residual), BasicTransformerBlock (LN->attn1, LN->attn2, LN->GEGLU FF,
  each + residual), Attention (8 heads, q/k/v no bias, to_out bias),
  Downsample2D (conv3x3 stride 2 pad 1), Upsample2D (nearest x2, conv3x3),
  skip concat cat([h, skip], dim=1).
The cross-attention is the reference processor, models/audio_attention_processor.py:
  :88  audio_projected = audio_proj(audio_tokens)    (Linear 768->64, GELU, Dropout, Linear 64->768)
  :94  audio_pooled = audio_projected.mean(dim=1, keepdim=True)
  :96  gate = sigmoid(alpha)
  :97  encoder_hidden_states = encoder_hidden_states + gate * audio_pooled
  :115-135 q = to_q(h)*scale; k,v = to_k/to_v(ehs); softmax(q k^T / sqrt(d)) v; to_out
and the level routing of AudioProcessorManager._create_level_mapping (:170-191).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def level_of(block_name: str) -> str:
    """AudioProcessorManager._create_level_mapping (reference :179-191)."""
    if "mid_block" in block_name:
        return "mid"
    if "down_blocks.0" in block_name or "down_blocks.1" in block_name:
        return "early"
    if "down_blocks.2" in block_name or "down_blocks.3" in block_name:
        return "late"
    if "up_blocks.0" in block_name or "up_blocks.1" in block_name:
        return "late"
    if "up_blocks.2" in block_name or "up_blocks.3" in block_name:
        return "mid"
    return "mid"


def timestep_embedding(t: torch.Tensor, dim: int = 320) -> torch.Tensor:
    half = dim // 2
    exponent = -math.log(10000) * torch.arange(half, dtype=torch.float32) / half
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    return torch.cat([emb[:, half:], emb[:, :half]], dim=-1)  # flip_sin_to_cos


def processor_call(w: dict, proc_w: dict | None, h: torch.Tensor, ehs: torch.Tensor | None, audio: dict | None,
                   level: str, heads: int = 8, mask: torch.Tensor | None = None, scale: float = 1.0,
                   mode: str = "add") -> torch.Tensor:
    """The reference AudioAttnProcessor.__call__ (models/audio_attention_processor.py:62-145) on
    an Attention with weights w (to_q / to_k / to_v / to_out.0), fp32:
      :67-70   4-D [B, C, H, W] input viewed as [B, H*W, C]
      :86-109  audio injection only when encoder_hidden_states is given (Add-FiLM or concat)
      :115-121 q = to_q(h) * scale; with no encoder_hidden_states, K / V come from that
               projected query (encoder_hidden_states = hidden_states after :115)
      :129     get_attention_scores: baddbmm(mask, q, k^T, beta=1, alpha=d^-0.5), softmax
      :137-138 output transposed back to [B, C, H, W]."""
    nd4 = h.dim() == 4
    if nd4:
        b, c, hh, ww = h.shape
        h = h.reshape(b, c, hh * ww).transpose(1, 2)
    if ehs is not None and audio is not None and level in audio and proc_w is not None:
        a = F.linear(audio[level].float(), proc_w["audio_proj.0.weight"], proc_w["audio_proj.0.bias"])
        a = F.linear(F.gelu(a), proc_w["audio_proj.3.weight"], proc_w["audio_proj.3.bias"])
        if mode == "add":
            ehs = ehs + torch.sigmoid(proc_w["alpha"].float()) * a.mean(dim=1, keepdim=True)
        else:
            if a.shape[1] > 4:
                a = F.adaptive_avg_pool1d(a.transpose(1, 2), 4).transpose(1, 2)
            ehs = torch.cat([ehs, a], dim=1)
    q = F.linear(h, w["to_q.weight"]) * scale
    ctx = q if ehs is None else ehs
    k, v = F.linear(ctx, w["to_k.weight"]), F.linear(ctx, w["to_v.weight"])
    b, lq, inner = q.shape
    d = inner // heads

    def hb(t):
        return t.reshape(b, t.shape[1], heads, d).permute(0, 2, 1, 3).reshape(b * heads, t.shape[1], d)
    s = torch.bmm(hb(q), hb(k).transpose(1, 2)) * d ** -0.5
    if mask is not None:
        s = s + mask
    o = torch.bmm(s.softmax(-1), hb(v)).reshape(b, heads, lq, d).permute(0, 2, 1, 3).reshape(b, lq, inner)
    o = F.linear(o, w["to_out.0.weight"], w.get("to_out.0.bias"))
    if nd4:
        o = o.transpose(-1, -2).reshape(b, c, hh, ww)
    return o


class UNetRef:
    def __init__(self, sd: dict, processors: dict | None = None, heads: int = 8, groups: int = 32):
        self.sd = {k: v.float() for k, v in sd.items()}
        self.proc = processors or {}
        self.heads = heads
        self.groups = groups

    def p(self, k):
        return self.sd[k]

    def conv(self, pre, x, stride=1):
        w = self.p(pre + ".weight")
        return F.conv2d(x, w, self.p(pre + ".bias"), stride=stride, padding=w.shape[-1] // 2)

    def gn(self, pre, x, eps):
        return F.group_norm(x, self.groups, self.p(pre + ".weight"), self.p(pre + ".bias"), eps)

    def lin(self, pre, x):
        return F.linear(x, self.p(pre + ".weight"), self.sd.get(pre + ".bias"))

    def ln(self, pre, x):
        return F.layer_norm(x, (x.shape[-1],), self.p(pre + ".weight"), self.p(pre + ".bias"), 1e-5)

    def resnet(self, pre, x, temb):
        h = self.conv(pre + ".conv1", F.silu(self.gn(pre + ".norm1", x, 1e-5)))
        h = h + self.lin(pre + ".time_emb_proj", F.silu(temb))[:, :, None, None]
        h = self.conv(pre + ".conv2", F.silu(self.gn(pre + ".norm2", h, 1e-5)))
        if pre + ".conv_shortcut.weight" in self.sd:
            x = self.conv(pre + ".conv_shortcut", x)
        return x + h

    def attention(self, pre, x, ctx, bias=None):
        """bias: additive score bias broadcast to [b, heads, lq, lk] (diffusers
        get_attention_scores adds attention_mask to q k^T * scale)."""
        c = x.shape[-1]
        h = self.heads
        d = c // h
        q = self.lin(pre + ".to_q", x)
        k = self.lin(pre + ".to_k", ctx)
        v = self.lin(pre + ".to_v", ctx)
        b, lq, _ = q.shape
        lk = k.shape[1]
        q = q.view(b, lq, h, d).transpose(1, 2)
        k = k.view(b, lk, h, d).transpose(1, 2)
        v = v.view(b, lk, h, d).transpose(1, 2)
        o = torch.empty_like(q)
        for i in range(0, lq, 2048):   # query blocks: bounded score memory at 96^2 (c5)
            s = torch.matmul(q[:, :, i:i + 2048], k.transpose(-1, -2)) * (d ** -0.5)
            if bias is not None:
                s = s + bias
            o[:, :, i:i + 2048] = torch.matmul(s.softmax(-1), v)
        o = o.transpose(1, 2).reshape(b, lq, c)
        return self.lin(pre + ".to_out.0", o)

    def audio_context(self, level: str, ehs: torch.Tensor, audio: dict | None) -> torch.Tensor:
        """reference processor :76-97 (Add-FiLM branch)."""
        if audio is None or level not in audio or level not in self.proc:
            return ehs
        w = self.proc[level]
        a = audio[level].float()
        a = F.linear(a, w["audio_proj.0.weight"], w["audio_proj.0.bias"])
        a = F.gelu(a)
        a = F.linear(a, w["audio_proj.3.weight"], w["audio_proj.3.bias"])
        pooled = a.mean(dim=1, keepdim=True)
        gate = torch.sigmoid(w["alpha"].float())
        return ehs + gate * pooled

    def transformer(self, pre, x, ehs, audio, mask_bias=None):
        b, c, hh, ww = x.shape
        res = x
        h = self.conv(pre + ".proj_in", self.gn(pre + ".norm", x, 1e-6))
        h = h.permute(0, 2, 3, 1).reshape(b, hh * ww, c)
        blk = pre + ".transformer_blocks.0"
        n = self.ln(blk + ".norm1", h)
        h = self.attention(blk + ".attn1", n, n) + h
        n = self.ln(blk + ".norm2", h)
        ctx = self.audio_context(level_of(pre), ehs, audio)
        h = self.attention(blk + ".attn2", n, ctx, mask_bias) + h
        n = self.ln(blk + ".norm3", h)
        hid, gate = self.lin(blk + ".ff.net.0.proj", n).chunk(2, dim=-1)
        h = self.lin(blk + ".ff.net.2", hid * F.gelu(gate)) + h
        h = h.reshape(b, hh, ww, c).permute(0, 3, 1, 2)
        return self.conv(pre + ".proj_out", h) + res

    def __call__(self, sample, t, ehs, audio=None, encoder_attention_mask=None):
        """sample [N,4,H,W] fp32, t scalar or [N], ehs [N,77,768], audio {level: [N,K,768]};
        encoder_attention_mask [N, 77] keep-mask -> (1 - m) * -10000 bias on every attn2
        (diffusers 0.23.1 UNet2DConditionModel.forward)."""
        n = sample.shape[0]
        mb = None
        if encoder_attention_mask is not None:
            mb = ((1.0 - encoder_attention_mask.float()) * -10000.0)[:, None, None, :]
        t = torch.as_tensor(t, dtype=torch.float32).reshape(-1).expand(n)
        temb = timestep_embedding(t, self.p("conv_in.weight").shape[0])
        temb = self.lin("time_embedding.linear_2", F.silu(self.lin("time_embedding.linear_1", temb)))
        h = self.conv("conv_in", sample.float())
        skips = [h]
        nblocks = 4
        for i in range(nblocks):
            for j in range(2):
                h = self.resnet(f"down_blocks.{i}.resnets.{j}", h, temb)
                if f"down_blocks.{i}.attentions.{j}.norm.weight" in self.sd:
                    h = self.transformer(f"down_blocks.{i}.attentions.{j}", h, ehs, audio, mb)
                skips.append(h)
            if f"down_blocks.{i}.downsamplers.0.conv.weight" in self.sd:
                h = self.conv(f"down_blocks.{i}.downsamplers.0.conv", h, stride=2)
                skips.append(h)
        h = self.resnet("mid_block.resnets.0", h, temb)
        h = self.transformer("mid_block.attentions.0", h, ehs, audio, mb)
        h = self.resnet("mid_block.resnets.1", h, temb)
        for i in range(nblocks):
            for j in range(3):
                h = torch.cat([h, skips.pop()], dim=1)
                h = self.resnet(f"up_blocks.{i}.resnets.{j}", h, temb)
                if f"up_blocks.{i}.attentions.{j}.norm.weight" in self.sd:
                    h = self.transformer(f"up_blocks.{i}.attentions.{j}", h, ehs, audio, mb)
            if f"up_blocks.{i}.upsamplers.0.conv.weight" in self.sd:
                h = F.interpolate(h, scale_factor=2.0, mode="nearest")
                h = self.conv(f"up_blocks.{i}.upsamplers.0.conv", h)
        h = F.silu(self.gn("conv_norm_out", h, 1e-5))
        return self.conv("conv_out", h)
