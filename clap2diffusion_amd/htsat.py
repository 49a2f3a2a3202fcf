"""CLAP HTSAT audio tower on the HIP kernels (fp16 activations, fp32 accumulate).

Replaces transformers ClapModel.get_audio_features (htsat-unfused), called by
the reference CLAPAudioEncoder.encode_audio (models/audio_encoder.py:171-174):
  c2d_htsat_mel_patches   BatchNorm over mel bins + bicubic 1001->1024 + mel->image fold + 4x4 patches
  GEMM                    patch-embed conv (as a K=16 GEMM), then LayerNorm (apply kernel)
  per Swin block          LN-prologue fused QKV GEMM -> c2d_window_attention (cyclic shift,
                          window partition and reverse folded into a row map; relative-position
                          bias + shift mask) -> dense GEMM (+ residual) -> LN-prologue GEMM + GELU
                          -> GEMM (+ residual)
  patch merging           gather kernel -> LN-prologue reduction GEMM
  head                    final LayerNorm -> token mean -> Linear+ReLU -> Linear -> L2 normalise
Weights load from ClapModel-keyed state dicts (audio_model.audio_encoder.*, audio_projection.*).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .layers import HLayerNorm, HLinear
from .weights import HTSAT_CFG

E = "audio_model.audio_encoder."


def _rel_index(w: int) -> np.ndarray:
    ys, xs = np.meshgrid(np.arange(w), np.arange(w), indexing="ij")
    c = np.stack([ys.ravel(), xs.ravel()])
    rel = (c[:, :, None] - c[:, None, :]).transpose(1, 2, 0) + (w - 1)
    return rel[..., 0] * (2 * w - 1) + rel[..., 1]


def _row_map(b: int, h: int, w: int, win: int, shift: int) -> np.ndarray:
    """window-ordered token -> row of the [b*h*w] token matrix (roll by -shift, partition)."""
    wy, wx, ty, tx = np.meshgrid(np.arange(h // win), np.arange(w // win), np.arange(win), np.arange(win),
                                 indexing="ij")
    y = (wy * win + ty + shift) % h
    x = (wx * win + tx + shift) % w
    per_img = (y * w + x).reshape(-1)
    return (np.arange(b)[:, None] * (h * w) + per_img[None, :]).reshape(-1).astype(np.int32)


def _shift_mask(h: int, w: int, win: int, shift: int) -> np.ndarray:
    def region(n):
        i = np.arange(n)
        return (i >= n - win).astype(np.int64) + (i >= n - shift).astype(np.int64)
    lab = region(h)[:, None] * 3 + region(w)[None, :]
    lab = lab.reshape(h // win, win, w // win, win).transpose(0, 2, 1, 3).reshape(-1, win * win)
    m = lab[:, None, :] - lab[:, :, None]
    return np.where(m != 0, -100.0, 0.0).astype(np.float32)


class SwinBlock(nn.Module):
    def __init__(self, dim: int, heads: int, mlp: int):
        super().__init__()
        self.dim, self.heads = dim, heads
        self.layernorm_before = HLayerNorm(dim)
        self.qkv = HLinear(dim, 3 * dim)
        self.dense = HLinear(dim, dim)
        self.layernorm_after = HLayerNorm(dim)
        self.intermediate = HLinear(dim, mlp * dim)
        self.output = HLinear(mlp * dim, dim)
        self.register_buffer("bias_table", torch.zeros(heads, 64, 64), persistent=False)

    def forward(self, x, row_map, mask, n_windows):
        qkv = self.qkv(x, ln=self.layernorm_before.prologue(x))
        att = torch.empty_like(x)
        ops.window_attention(qkv, row_map, n_windows, self.heads, self.dim // self.heads, self.bias_table, mask, att)
        x = self.dense(att, resid=x)
        h = self.intermediate(x, ln=self.layernorm_after.prologue(x), act="gelu")
        return self.output(h, resid=x, out=x)


class HTSATEncoder(nn.Module):
    """mel [B, T, 64] fp32 (T <= 1024) -> L2-normalised CLAP audio embedding [B, 512] fp32."""

    def __init__(self, cfg: dict = HTSAT_CFG):
        super().__init__()
        self.cfg = dict(cfg)
        emb = cfg["embed"]
        self.patch_proj = HLinear(16, emb)
        self.patch_norm = HLayerNorm(emb)
        self.stages = nn.ModuleList()
        self.merges = nn.ModuleList()
        for i, depth in enumerate(cfg["depths"]):
            dim = emb * 2 ** i
            self.stages.append(nn.ModuleList([SwinBlock(dim, cfg["heads"][i], cfg["mlp_ratio"]) for _ in range(depth)]))
            if i < len(cfg["depths"]) - 1:
                m = nn.Module()
                m.norm = HLayerNorm(4 * dim)
                m.reduction = HLinear(4 * dim, 2 * dim, bias=False)
                self.merges.append(m)
        self.norm = HLayerNorm(cfg["hidden"])
        self.linear1 = HLinear(cfg["hidden"], cfg["proj_dim"])
        self.linear2 = HLinear(cfg["proj_dim"], cfg["proj_dim"])
        self.register_buffer("bn_scale", torch.ones(cfg["mel_bins"]), persistent=False)
        self.register_buffer("bn_shift", torch.zeros(cfg["mel_bins"]), persistent=False)
        self._maps = {}

    @torch.no_grad()
    def load_clap_state_dict(self, sd: dict) -> None:
        g = lambda k: sd[k].float()  # noqa: E731
        bn_w, bn_b = g(E + "batch_norm.weight"), g(E + "batch_norm.bias")
        rm, rv = g(E + "batch_norm.running_mean"), g(E + "batch_norm.running_var")
        sc = bn_w / torch.sqrt(rv + 1e-5)
        self.bn_scale.copy_(sc)
        self.bn_shift.copy_(bn_b - rm * sc)
        self.patch_proj.load(g(E + "patch_embed.proj.weight").reshape(self.cfg["embed"], 16),
                             g(E + "patch_embed.proj.bias"))
        self.patch_norm.load(g(E + "patch_embed.norm.weight"), g(E + "patch_embed.norm.bias"))
        idx = torch.from_numpy(_rel_index(self.cfg["window"]).reshape(-1))
        for i, stage in enumerate(self.stages):
            for j, blk in enumerate(stage):
                k = f"{E}layers.{i}.blocks.{j}."
                blk.layernorm_before.load(g(k + "layernorm_before.weight"), g(k + "layernorm_before.bias"))
                blk.qkv.load(torch.cat([g(f"{k}attention.self.{n}.weight") for n in ("query", "key", "value")]),
                             torch.cat([g(f"{k}attention.self.{n}.bias") for n in ("query", "key", "value")]))
                blk.dense.load(g(k + "attention.output.dense.weight"), g(k + "attention.output.dense.bias"))
                blk.layernorm_after.load(g(k + "layernorm_after.weight"), g(k + "layernorm_after.bias"))
                blk.intermediate.load(g(k + "intermediate.dense.weight"), g(k + "intermediate.dense.bias"))
                blk.output.load(g(k + "output.dense.weight"), g(k + "output.dense.bias"))
                tab = g(k + "attention.self.relative_position_bias_table")
                blk.bias_table.copy_(tab[idx].view(64, 64, -1).permute(2, 0, 1))
            if i < len(self.stages) - 1:
                k = f"{E}layers.{i}.downsample."
                self.merges[i].norm.load(g(k + "norm.weight"), g(k + "norm.bias"))
                self.merges[i].reduction.load(g(k + "reduction.weight"))
        self.norm.load(g(E + "norm.weight"), g(E + "norm.bias"))
        self.linear1.load(g("audio_projection.linear1.weight"), g("audio_projection.linear1.bias"))
        self.linear2.load(g("audio_projection.linear2.weight"), g("audio_projection.linear2.bias"))

    def _window_tables(self, b: int, device):
        key = (b, str(device))
        if key not in self._maps:
            tabs = []
            h, win = 64, self.cfg["window"]
            for i, depth in enumerate(self.cfg["depths"]):
                per = []
                for j in range(depth):
                    w_eff = min(win, h)
                    shift = 0 if (j % 2 == 0 or h <= win) else win // 2
                    rm = torch.from_numpy(_row_map(b, h, h, w_eff, shift)).to(device)
                    mask = torch.from_numpy(_shift_mask(h, h, w_eff, shift)).to(device) if shift else None
                    per.append((rm, mask, b * (h // w_eff) ** 2))
                tabs.append(per)
                h //= 2
            self._maps[key] = tabs
        return self._maps[key]

    @torch.no_grad()
    def forward(self, mel: torch.Tensor) -> torch.Tensor:
        if mel.dim() == 4:
            mel = mel[:, 0]
        mel = mel.float().contiguous()
        b = mel.shape[0]
        tabs = self._window_tables(b, mel.device)
        p = ops.htsat_mel_patches(mel, self.bn_scale, self.bn_shift)
        x = self.patch_norm(self.patch_proj(p))  # K = 64 with 16 live columns
        h = 64
        for i, stage in enumerate(self.stages):
            for j, blk in enumerate(stage):
                rm, mask, nw = tabs[i][j]
                x = blk(x, rm, mask, nw)
            if i < len(self.stages) - 1:
                c = x.shape[1]
                m = ops.patch_merge_gather(x, b, h, h, c)
                x = self.merges[i].reduction(m, ln=self.merges[i].norm.prologue(m))
                h //= 2
        y = self.norm(x)
        pooled = ops.row_mean(y, b, h * h).to(torch.float16)
        z = self.linear2(self.linear1(pooled, act="relu"))
        return ops.l2_normalize_(z.float().contiguous())
