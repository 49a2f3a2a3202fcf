"""fp32 CPU restatement of the CLAP HTSAT audio tower (TEST ORACLE ONLY).

Restates transformers ClapModel.get_audio_features for the htsat-unfused
config (enable_fusion False), i.e. what the reference calls at
models/audio_encoder.py:171-174:
  ClapAudioEncoder.forward      modeling_clap.py:798-902 (BatchNorm over mel bins,
                                reshape_mel2img :761-798, patch embed + LN, 4 Swin stages,
                                final LN, token mean pool)
  ClapAudioLayer / SelfAttention :323-414, :504-621 (cyclic shift, window partition,
                                relative-position bias, shift mask -100, window reverse)
  ClapAudioPatchMerging          :680-717
  ClapProjectionLayer            :905-921, then F.normalize (:1533)
Pinned against tests/golden/htsat.npz (generated from transformers ClapModel).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

DEPTHS, HEADS, WINDOW = (2, 2, 6, 2), (4, 8, 16, 32), 8


def relative_position_index(w: int = WINDOW) -> torch.Tensor:
    ys, xs = np.meshgrid(np.arange(w), np.arange(w), indexing="ij")
    c = np.stack([ys.ravel(), xs.ravel()])
    rel = (c[:, :, None] - c[:, None, :]).transpose(1, 2, 0) + (w - 1)
    return torch.from_numpy(rel[..., 0] * (2 * w - 1) + rel[..., 1])


def shift_mask(h: int, w: int, win: int, shift: int) -> torch.Tensor:
    """[nW, win*win, win*win] with 0 / -100 (ClapAudioLayer.get_attn_mask)."""
    def region(n):
        i = np.arange(n)
        return (i >= n - win).astype(np.int64) + (i >= n - shift).astype(np.int64)
    lab = region(h)[:, None] * 3 + region(w)[None, :]
    lab = lab.reshape(h // win, win, w // win, win).transpose(0, 2, 1, 3).reshape(-1, win * win)
    m = lab[:, None, :] - lab[:, :, None]
    return torch.from_numpy(np.where(m != 0, -100.0, 0.0).astype(np.float32))


def _ln(x, sd, k, eps=1e-5):
    return F.layer_norm(x, (x.shape[-1],), sd[k + ".weight"], sd[k + ".bias"], eps)


def _lin(x, sd, k):
    return F.linear(x, sd[k + ".weight"], sd.get(k + ".bias"))


def swin_block(x, sd, k, b, h, w, c, heads, shift):
    win = WINDOW
    if min(h, w) <= win:
        shift, win = 0, min(h, w)
    short = x
    y = _ln(x, sd, k + ".layernorm_before").view(b, h, w, c)
    if shift:
        y = torch.roll(y, (-shift, -shift), (1, 2))
    y = y.view(b, h // win, win, w // win, win, c).permute(0, 1, 3, 2, 4, 5).reshape(-1, win * win, c)
    nw = y.shape[0]
    d = c // heads
    q = _lin(y, sd, k + ".attention.self.query").view(nw, -1, heads, d).transpose(1, 2)
    kk = _lin(y, sd, k + ".attention.self.key").view(nw, -1, heads, d).transpose(1, 2)
    v = _lin(y, sd, k + ".attention.self.value").view(nw, -1, heads, d).transpose(1, 2)
    s = q @ kk.transpose(-1, -2) / d ** 0.5
    table = sd[k + ".attention.self.relative_position_bias_table"]
    bias = table[relative_position_index(win).reshape(-1)].view(win * win, win * win, heads).permute(2, 0, 1)
    s = s + bias.unsqueeze(0)
    if shift:
        m = shift_mask(h, w, win, shift)
        s = (s.view(b, m.shape[0], heads, win * win, win * win) + m[None, :, None]).view(nw, heads, win * win, -1)
    o = (s.softmax(-1) @ v).transpose(1, 2).reshape(nw, win * win, c)
    o = _lin(o, sd, k + ".attention.output.dense")
    o = o.view(b, h // win, w // win, win, win, c).permute(0, 1, 3, 2, 4, 5).reshape(b, h, w, c)
    if shift:
        o = torch.roll(o, (shift, shift), (1, 2))
    x = short + o.reshape(b, h * w, c)
    m = F.gelu(_lin(_ln(x, sd, k + ".layernorm_after"), sd, k + ".intermediate.dense"))
    return x + _lin(m, sd, k + ".output.dense")


def patch_merge(x, sd, k, b, h, w, c):
    x = x.view(b, h, w, c)
    x = torch.cat([x[:, r::2, cc::2, :] for cc in range(2) for r in range(2)], dim=-1).view(b, -1, 4 * c)
    return F.linear(_ln(x, sd, k + ".norm"), sd[k + ".reduction.weight"])


def htsat_forward(sd: dict, mel: torch.Tensor, return_pooled: bool = False) -> torch.Tensor:
    """mel: [B, 1, T, 64] fp32 log-mel (ClapFeatureExtractor layout) -> [B, 512] L2-normalised."""
    sd = {k: v.float() for k, v in sd.items()}
    e = "audio_model.audio_encoder."
    x = mel.float()[:, 0]
    b, t, f = x.shape
    x = (x - sd[e + "batch_norm.running_mean"]) / torch.sqrt(sd[e + "batch_norm.running_var"] + 1e-5) \
        * sd[e + "batch_norm.weight"] + sd[e + "batch_norm.bias"]
    if t < 1024:
        x = F.interpolate(x[:, None], (1024, f), mode="bicubic", align_corners=True)[:, 0]
    img = x.reshape(b, 4, 256, f).permute(0, 1, 3, 2).reshape(b, 1, 4 * f, 256)
    x = F.conv2d(img, sd[e + "patch_embed.proj.weight"], sd[e + "patch_embed.proj.bias"], stride=4)
    x = _ln(x.flatten(2).transpose(1, 2), sd, e + "patch_embed.norm")
    h = w = 64
    c = x.shape[-1]
    for i, depth in enumerate(DEPTHS):
        for j in range(depth):
            x = swin_block(x, sd, f"{e}layers.{i}.blocks.{j}", b, h, w, c, HEADS[i], 0 if j % 2 == 0 else WINDOW // 2)
        if i < len(DEPTHS) - 1:
            x = patch_merge(x, sd, f"{e}layers.{i}.downsample", b, h, w, c)
            h, w, c = h // 2, w // 2, 2 * c
    pooled = _ln(x, sd, e + "norm").mean(dim=1)
    if return_pooled:
        return pooled
    y = F.linear(F.relu(F.linear(pooled, sd["audio_projection.linear1.weight"], sd["audio_projection.linear1.bias"])),
                 sd["audio_projection.linear2.weight"], sd["audio_projection.linear2.bias"])
    return F.normalize(y, dim=-1)
