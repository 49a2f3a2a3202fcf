"""Leaf layers holding packed fp16 weights for the HIP kernels.

Each layer keeps the parameter *names* of its torch / diffusers counterpart
(weight, bias) so checkpoint keys map 1:1, but stores the weight pre-packed
for the implicit-GEMM kernel (fp16 [out][kpad], K ordered (ky, kx, cin)) and
the bias in fp32.  Calling a layer runs the HIP kernel; there is no torch
compute fallback.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops


class HLinear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.kpad = ops.kpad_of(in_features)
        self.register_buffer("weight", torch.zeros(out_features, self.kpad, dtype=torch.float16))
        self.register_buffer("bias", torch.zeros(out_features, dtype=torch.float32) if bias else None)

    @torch.no_grad()
    def load(self, w: torch.Tensor, b: torch.Tensor | None = None) -> None:
        wp, kp = ops.pack_linear_weight(w.float())
        assert kp == self.kpad and wp.shape[0] == self.out_features
        self.weight.copy_(wp)
        if self.bias is not None:
            self.bias.copy_(b.float() if b is not None else torch.zeros_like(self.bias))

    def forward(self, x: torch.Tensor, **kw) -> torch.Tensor:
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        out = ops.conv(x2, self.weight, self.kpad, self.out_features, ksize=1, bias=self.bias, **kw)
        return out.view(*shp[:-1], out.shape[-1])


class HConv2d(nn.Module):
    """NHWC conv (ksize 1 or 3, pad = ksize // 2) on the implicit-GEMM kernel."""

    def __init__(self, cin: int, cout: int, ksize: int, stride: int = 1, cin_pad: int | None = None):
        super().__init__()
        self.cin, self.cout, self.ksize, self.stride = cin, cout, ksize, stride
        self.cin_pad = cin_pad or cin
        self.kpad = ops.kpad_of(ksize * ksize * self.cin_pad)
        self.register_buffer("weight", torch.zeros(cout, self.kpad, dtype=torch.float16))
        self.register_buffer("bias", torch.zeros(cout, dtype=torch.float32))

    @torch.no_grad()
    def load(self, w: torch.Tensor, b: torch.Tensor | None) -> None:
        wp, kp = ops.pack_conv_weight(w.float(), cin_pad=self.cin_pad if self.cin_pad != self.cin else None)
        assert kp == self.kpad, (kp, self.kpad)
        self.weight.copy_(wp)
        if b is not None:
            self.bias.copy_(b.float())

    def forward(self, x: torch.Tensor, **kw) -> torch.Tensor:
        return ops.conv(x, self.weight, self.kpad, self.cout, ksize=self.ksize, stride=self.stride, bias=self.bias, **kw)


class HGroupNorm(nn.Module):
    """GroupNorm parameters; `stats(x)` returns the folded (scale, shift) tables
    consumed by the conv prologue (c2d_groupnorm_stats)."""

    def __init__(self, num_groups: int, num_channels: int, eps: float):
        super().__init__()
        self.num_groups, self.num_channels, self.eps = num_groups, num_channels, eps
        self.register_buffer("weight", torch.ones(num_channels))
        self.register_buffer("bias", torch.zeros(num_channels))

    @torch.no_grad()
    def load(self, w, b):
        self.weight.copy_(w.float())
        self.bias.copy_(b.float())

    def stats(self, x: torch.Tensor, x2: torch.Tensor | None = None):
        return ops.group_norm_stats(x, self.num_groups, self.eps, self.weight, self.bias, x2=x2)

    def apply(self, x: torch.Tensor, x2: torch.Tensor | None = None, silu: bool = False,
              pad: bool = False, mom=None) -> torch.Tensor:
        """act(GroupNorm(cat[x, x2])) materialised once (c2d_groupnorm); pad: in the zero-bordered
        layout a conv(..., padded=True) reads (c2d_groupnorm_pad); mom: x's moments from its producing
        conv (ops.GnMoments, c2d_groupnorm_moments), used when they match x and this norm's groups."""
        return ops.group_norm(x, self.num_groups, self.eps, self.weight, self.bias, silu, x2=x2, pad=pad, mom=mom)


class HLayerNorm(nn.Module):
    def __init__(self, c: int, eps: float = 1e-5):
        super().__init__()
        self.c, self.eps = c, eps
        self.register_buffer("weight", torch.ones(c))
        self.register_buffer("bias", torch.zeros(c))

    @torch.no_grad()
    def load(self, w, b):
        self.weight.copy_(w.float())
        self.bias.copy_(b.float())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        return ops.layer_norm(x.reshape(-1, shp[-1]), self.weight, self.bias, self.eps).view(shp)

    def prologue(self, x2d: torch.Tensor):
        """(stats, gamma, beta) for a C2D_PRO_LN GEMM prologue."""
        return ops.layer_norm_stats(x2d, self.eps), self.weight, self.bias


def load_tree(module: nn.Module, sd: dict, prefix: str = "") -> list[str]:
    """Load a diffusers/transformers-keyed state dict into a tree of H* layers.
    Returns the list of consumed keys."""
    used = []
    for name, m in module.named_modules():
        if isinstance(m, (HLinear, HConv2d, HGroupNorm, HLayerNorm)):
            key = (prefix + name) if name else prefix.rstrip(".")
            wk, bk = key + ".weight", key + ".bias"
            if wk not in sd:
                raise KeyError(f"missing weight {wk}")
            m.load(sd[wk], sd.get(bk))
            used.append(wk)
            if bk in sd:
                used.append(bk)
    return used
