"""Torch-facing API over the C ABI (include/c2d.h), through the torch.library ops.

Tensors are plain device buffers here: activations NHWC / row-major fp16,
statistics fp32.  Each function checks its operands, allocates the outputs and
calls the registered ``torch.ops.c2d.*`` operator (clap2diffusion_amd.torch_ops),
whose CUDA implementation launches the HIP kernel on torch's current stream, so
the calls can be captured into a torch.cuda.CUDAGraph (hipGraph) as is.
"""
from __future__ import annotations

import ctypes
import functools
import math

import torch

from . import torch_ops  # noqa: F401  (registers the c2d:: operators)
from ._lib import C2D_ACT

C2D = torch.ops.c2d

F16 = torch.float16


def _require(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a device tensor (HIP path only, no CPU fallback)")


# ----------------------------------------------------------------- packing
def kpad_of(k: int) -> int:
    return (k + 63) // 64 * 64


def pack_conv_weight(w: torch.Tensor, cin_pad: int | None = None) -> tuple[torch.Tensor, int]:
    """[cout, cin, kh, kw] -> fp16 [cout][kpad] with K ordered (ky, kx, cin)."""
    cout, cin, kh, kw = w.shape
    if cin_pad and cin_pad > cin:
        w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, cin_pad - cin))
        cin = cin_pad
    k = kh * kw * cin
    wp = w.permute(0, 2, 3, 1).reshape(cout, k)
    kp = kpad_of(k)
    if kp > k:
        wp = torch.nn.functional.pad(wp, (0, kp - k))
    return wp.to(F16).contiguous(), kp


def pack_weights_device(w: torch.Tensor, cin_pad: int | None = None) -> tuple[torch.Tensor, int]:
    """c2d_pack_weights: the on-device form of pack_conv_weight / pack_linear_weight
    (fp32 weight already on the GPU -> fp16 [cout][kpad])."""
    _require(w, "w")
    w = w.float().contiguous()
    cout, cin = w.shape[:2]
    ks = w.shape[2] if w.dim() == 4 else 1
    cp = max(cin_pad or cin, cin)
    kp = kpad_of(ks * ks * cp)
    out = torch.empty(cout, kp, device=w.device, dtype=F16)
    C2D.pack_weights(w, cout, cin, ks, cp, kp, out)
    return out, kp


def pack_linear_weight(w: torch.Tensor) -> tuple[torch.Tensor, int]:
    """[out, in] -> fp16 [out][kpad]."""
    out_f, in_f = w.shape
    kp = kpad_of(in_f)
    wp = torch.nn.functional.pad(w, (0, kp - in_f)) if kp > in_f else w
    return wp.to(F16).contiguous(), kp


def geglu_interleave(w: torch.Tensor, b: torch.Tensor | None):
    """GEGLU proj [2I, in] (rows: h then g, diffusers chunk(2, -1)) -> rows in
    32-row blocks [h(16) | g(16)] so one MFMA column tile pair yields h*gelu(g)."""
    two_i = w.shape[0]
    inner = two_i // 2
    assert inner % 16 == 0
    idx = torch.arange(two_i).view(2, inner // 16, 16).permute(1, 0, 2).reshape(-1)
    wi = w[idx]
    bi = b[idx] if b is not None else None
    return wi, bi


# ----------------------------------------------------------------- kernels
def conv(x: torch.Tensor, weight: torch.Tensor, kpad: int, cout: int, *, ksize: int, bias=None, stride: int = 1,
         up: bool = False, x2: torch.Tensor | None = None, gn=None, gn_silu: bool = False, ln=None,
         silu_in: bool = False, act: str | None = None, temb: torch.Tensor | None = None,
         resid: torch.Tensor | None = None, out: torch.Tensor | None = None, padded: bool = False,
         ln_fold=None, gn_moments: int = 0):
    """Implicit-GEMM conv / linear (c2d::conv2d_igemm).

    x: NHWC [N, H, W, C0] fp16 (or 2-D [M, C0] for a linear layer); padded: x is the
    zero-bordered [N, H + 2, W + 2, C0] of group_norm(pad=True) (3x3, stride 1, one source).
    gn: (scale, shift) fp32 [N, C0+C1]; ln: (stats [M, 2], gamma, beta).
    ln_fold: eps of a LayerNorm folded into this linear: x is the LayerNorm's raw input
    (weight = W diag(gamma), bias = b + W beta; fold_layernorm builds them), panel GEMM shapes only.
    gn_moments = G > 0: also have the conv emit the GroupNorm moments of its output over G groups
    where the library can (c2d_conv2d_gn_rows); returns (out, GnMoments or None) instead of out.
    """
    _require(x, "x")
    if x.dim() == 2:
        h, w = 1, x.shape[0]
    else:
        _, h, w, _ = x.shape
        if padded:
            assert ksize == 3 and stride == 1 and not up and x2 is None, "padded source: 3x3, stride 1, one source"
            # the zero border is data to the kernels (pad 0): a prologue would map it to shift / SiLU(shift)
            assert gn is None and ln is None and not silu_in, "padded source: no GN / LN / SiLU prologue"
            h, w = h - 2, w - 2
    assert x.is_contiguous() and x.dtype == F16
    if x2 is not None:
        assert x2.is_contiguous() and x2.dtype == F16 and x2.shape[:-1] == x.shape[:-1]
    if ksize == 3:
        vh, vw = (2 * h, 2 * w) if up else (h, w)
        oh, ow = (vh + 2 - 3) // stride + 1, (vw + 2 - 3) // stride + 1
    else:
        oh, ow = h, w
    out_cols = cout // 2 if act == "geglu" else cout
    if out is None:
        shape = (x.shape[0], out_cols) if x.dim() == 2 else (x.shape[0], oh, ow, out_cols)
        out = torch.empty(shape, device=x.device, dtype=F16)
    assert out.stride(-1) == 1
    if resid is not None:
        assert resid.stride(-1) == 1
    gs, gh = gn if gn is not None else (None, None)
    ls, lg, lb = ln if ln is not None else (None, None, None)
    mom, rows = None, 0
    if gn_moments and x.dim() == 4 and act is None and not up and out.is_contiguous():
        rows = gn_moment_rows(out.shape[0], oh, ow, x.shape[-1], cout, ksize, stride, bool(padded), resid is not None,
                              temb is not None, gn_moments, x2.shape[-1] if x2 is not None else 0)
        if rows:
            mom = torch.empty((out.shape[0], oh * ow // rows, gn_moments, 2), device=x.device, dtype=torch.float32)
    C2D.conv2d_igemm(x, weight, kpad, cout, ksize, stride, up, x2, gs, gh, gn_silu, ls, lg, lb, silu_in, bias,
                     C2D_ACT[act], temb, resid, out, bool(padded), float(ln_fold or 0.0), mom, int(gn_moments))
    if gn_moments:
        return out, (GnMoments(out, mom, rows, gn_moments) if mom is not None else None)
    return out


class GnMoments:
    """GroupNorm moments a conv emitted for its output (c2d_conv_desc::gn_mom): mom fp32
    [N][H*W / rows][groups][2] of {mean, M2}; valid for `of` (that exact tensor) until it is written again."""

    def __init__(self, of: torch.Tensor, mom: torch.Tensor, rows: int, groups: int):
        self.of, self.mom, self.rows, self.groups = of, mom, rows, groups

    def matches(self, x: torch.Tensor, groups: int) -> bool:
        return (x is self.of and groups == self.groups and x.dim() == 4 and
                tuple(self.mom.shape[:1]) == tuple(x.shape[:1]))


@functools.lru_cache(maxsize=None)
def gn_moment_rows(n: int, oh: int, ow: int, cin: int, cout: int, ksize: int, stride: int, padded: bool, resid: bool,
                   temb: bool, groups: int, c1: int = 0) -> int:
    """c2d_conv2d_gn_rows for a conv of these shapes as ops.conv issues it (16-B aligned operands, a workspace
    for any split): rows per moment block, 0 = this conv cannot emit its output's GroupNorm moments."""
    import ctypes
    from ._lib import ConvDesc, lib
    d = ConvDesc()
    h, w = (oh, ow) if padded or ksize == 1 or stride == 1 else (oh * stride, ow * stride)
    d.c0, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride, d.src_pad = cin, n, h, w, oh, ow, ksize, stride, int(padded)
    d.c1 = c1
    if c1:
        d.src1 = 256
    d.cout, d.kpad, d.out_ld = cout, kpad_of(ksize * ksize * (cin + c1)), cout
    d.out = 256
    if resid:
        d.resid, d.resid_ld = 256, cout
    if temb:
        d.temb, d.temb_ld = 256, cout
    d.ws, d.ws_bytes = 256, 1 << 40
    d.gn_groups = groups
    return int(lib().c2d_conv2d_gn_rows(ctypes.byref(d)))


@torch.no_grad()
def fold_layernorm(weight: torch.Tensor, bias: torch.Tensor | None, gamma: torch.Tensor, beta: torch.Tensor,
                   in_features: int):
    """LayerNorm(gamma, beta) -> Linear(packed fp16 weight [cout][kpad], bias) as one GEMM over the
    normalised rows (C2D_PRO_LNFOLD): (W diag(gamma) fp16, b + W beta fp32)."""
    w = weight[:, :in_features].float()
    wp = torch.zeros_like(weight)
    wp[:, :in_features] = (w * gamma.float().view(1, -1)).to(F16)
    b = w @ beta.float()
    if bias is not None:
        b = b + bias.float()
    return wp.contiguous(), b.contiguous()


@functools.lru_cache(maxsize=None)
def panel_gemm(m: int, k: int, cout: int, geglu: bool, lnfold: bool = False) -> bool:
    """Does c2d's planner run this 1x1 GEMM (m x k -> cout) on the panel GEMM (tile 70)?  Where it
    does, a LayerNorm before it folds in.  lnfold: would the library take this GEMM with a folded
    LayerNorm (C2D_PRO_LNFOLD: the panel GEMM's shapes and switches, else C2D_E_SHAPE)?"""
    import ctypes
    from ._lib import C2D_PRO_LNFOLD, ConvDesc, lib
    d = ConvDesc()
    d.c0, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride = k, 1, 1, m, 1, m, 1, 1
    d.cout, d.kpad, d.act = cout, kpad_of(k), C2D_ACT["geglu" if geglu else None]
    d.out_ld = cout // 2 if geglu else cout
    if lnfold:
        d.pro, d.pro_eps = C2D_PRO_LNFOLD, 1e-5
    tid, ks = ctypes.c_int(), ctypes.c_int()
    rc = lib().c2d_conv2d_igemm_plan(ctypes.byref(d), ctypes.byref(tid), ctypes.byref(ks))
    return rc == 0 and tid.value == 70


ROWRING_TILES = (42, 43, 44)   # igemm_pp16r.h: output width 64 / 32 / 16


@functools.lru_cache(maxsize=None)
def rowring_conv(n: int, h: int, w: int, cin: int, cout: int) -> bool:
    """Does c2d's planner run a 3x3 stride-1 conv (n x h x w, cin -> cout) on a row-ring tile (42 / 43
    / 44, by output width) when its source is zero-bordered?  (Asked of the library, c2d_conv2d_igemm_plan: the padded
    layout is worth writing only where that kernel reads it.)"""
    import ctypes
    from ._lib import ConvDesc, check, lib
    d = ConvDesc()
    d.c0, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride = cin, n, h, w, h, w, 3, 1
    d.cout, d.kpad, d.src_pad = cout, kpad_of(9 * cin), 1
    d.out_ld = cout
    tid, ks = ctypes.c_int(), ctypes.c_int()
    check(lib().c2d_conv2d_igemm_plan(ctypes.byref(d), ctypes.byref(tid), ctypes.byref(ks)), "c2d_conv2d_igemm_plan")
    return tid.value in ROWRING_TILES


def conv_workspace_bytes(n: int, h: int, w: int, c0: int, c1: int, cout: int, ksize: int) -> int:
    """Split-K workspace c2d_conv2d_igemm asks for on a stride-1 conv (n x h x w, c0 [+ c1] -> cout),
    as torch_ops.conv2d_igemm allocates it (c2d_conv2d_igemm_workspace_size)."""
    import ctypes
    from ._lib import ConvDesc, lib
    d = ConvDesc()
    d.c0, d.c1, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride = c0, c1, n, h, w, h, w, ksize, 1
    d.cout, d.kpad, d.out_ld = cout, kpad_of(ksize * ksize * (c0 + c1)), cout
    return int(lib().c2d_conv2d_igemm_workspace_size(ctypes.byref(d)))


class record_conv_plans:
    """Context manager collecting the (tile_id, ksplit) plan of every conv call
    (c2d_conv2d_igemm_plan) -- lets tests assert which kernel configuration ran."""

    def __enter__(self):
        self.plans = []
        torch_ops._plan_probe = self.plans
        return self.plans

    def __exit__(self, *exc):
        torch_ops._plan_probe = None
        return False


class force_plan:
    """Context manager forcing the implicit-GEMM plan (tile id, K split; 0 = planner) through
    c2d_set_plan_override -- tests and tuning sweeps only, never the product path."""

    def __init__(self, tile: int, split: int = 0):
        self.tile, self.split = int(tile), int(split)

    def __enter__(self):
        import ctypes
        from ._lib import check, lib
        t, sp = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().c2d_get_plan_override(ctypes.byref(t), ctypes.byref(sp)), "c2d_get_plan_override")
        self.prev = (t.value, sp.value)   # restored on exit: nested overrides / env sweeps survive
        check(lib().c2d_set_plan_override(self.tile, self.split), "c2d_set_plan_override")
        rowring_conv.cache_clear()        # the planner's answers change under an override
        gn_moment_rows.cache_clear()
        return self

    def __exit__(self, *exc):
        from ._lib import lib
        lib().c2d_set_plan_override(*self.prev)
        rowring_conv.cache_clear()
        gn_moment_rows.cache_clear()
        return False


def plan_override_from_env() -> None:
    """Opt-in for the tuning scripts: C2D_GEMM_TILE / C2D_GEMM_SPLIT (environment) ->
    c2d_set_plan_override.  The library itself never reads them."""
    import os
    from ._lib import check, lib
    t, sp = int(os.environ.get("C2D_GEMM_TILE", "0") or 0), int(os.environ.get("C2D_GEMM_SPLIT", "0") or 0)
    if t or sp:
        check(lib().c2d_set_plan_override(t, sp), "c2d_set_plan_override")


def group_norm_stats(x: torch.Tensor, groups: int, eps: float, gamma: torch.Tensor, beta: torch.Tensor,
                     x2: torch.Tensor | None = None):
    """-> (scale, shift) fp32 [N, C] folding GroupNorm(groups, eps) + affine."""
    _require(x, "x")
    c = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    scale = torch.empty((x.shape[0], c), device=x.device, dtype=torch.float32)
    shift = torch.empty_like(scale)
    C2D.groupnorm_stats(x, x2, groups, float(eps), gamma, beta, scale, shift)
    return scale, shift


def group_norm_apply(x: torch.Tensor, gn, silu: bool, x2: torch.Tensor | None = None,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """Materialise act(GroupNorm(cat[x, x2])) from the folded (scale, shift) tables."""
    _require(x, "x")
    c = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    if out is None:
        out = torch.empty((*x.shape[:-1], c), device=x.device, dtype=F16)
    C2D.groupnorm_apply(x, x2, gn[0], gn[1], bool(silu), out)
    return out


def group_norm(x: torch.Tensor, groups: int, eps: float, gamma: torch.Tensor, beta: torch.Tensor, silu: bool,
               x2: torch.Tensor | None = None, out: torch.Tensor | None = None, pad: bool = False,
               mom: "GnMoments | None" = None) -> torch.Tensor:
    """act(GroupNorm(cat[x, x2])) in one c2d::groupnorm call (single fused kernel for
    small images, stats + apply otherwise).  pad: write the zero-bordered layout
    [N, H + 2, W + 2, C] (c2d::groupnorm_pad) for a conv(..., padded=True).  mom: the moments x's
    producing conv emitted (conv(..., gn_moments=groups)): one launch, no statistics pass."""
    _require(x, "x")
    c = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    if mom is not None and x2 is None and mom.matches(x, groups):
        n, h, w, _ = x.shape
        if out is None:
            out = torch.empty((n, h + 2, w + 2, c) if pad else x.shape, device=x.device, dtype=F16)
        C2D.groupnorm_moments(x, groups, float(eps), gamma, beta, bool(silu), mom.mom, mom.rows, bool(pad), out)
        return out
    if pad:
        n, h, w, _ = x.shape
        if out is None:
            out = torch.empty((n, h + 2, w + 2, c), device=x.device, dtype=F16)
        C2D.groupnorm_pad(x, x2, groups, float(eps), gamma, beta, bool(silu), out)
        return out
    if out is None:
        out = torch.empty((*x.shape[:-1], c), device=x.device, dtype=F16)
    C2D.groupnorm(x, x2, groups, float(eps), gamma, beta, bool(silu), out)
    return out


def layer_norm_stats(x2d: torch.Tensor, eps: float) -> torch.Tensor:
    _require(x2d, "x")
    st = torch.empty((x2d.shape[0], 2), device=x2d.device, dtype=torch.float32)
    C2D.layernorm_stats(x2d, float(eps), st)
    return st


def layer_norm(x2d: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float,
               out: torch.Tensor | None = None) -> torch.Tensor:
    _require(x2d, "x")
    if out is None:
        out = torch.empty(x2d.shape, device=x2d.device, dtype=F16)
    C2D.layernorm(x2d, gamma, beta, float(eps), out)
    return out


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, batch: int, heads: int, lq: int, lk: int,
              d: int, scale: float | None = None, out: torch.Tensor | None = None,
              key_bias: torch.Tensor | None = None) -> torch.Tensor:
    """q/k/v: 2-D row views [batch*L, >= heads*d] (column slices allowed).
    key_bias: optional additive score bias, fp32, either per key [batch|1, heads|1, lk]
    (c2d_attention_fwd_bias) or per (query, key) [batch|1, heads|1, lq|1, lk]
    (c2d_attention_fwd_mask); size-1 dims broadcast."""
    _require(q, "q")
    if scale is None:
        scale = 1.0 / math.sqrt(d)
    if out is None:
        out = torch.empty((batch * lq, heads * d), device=q.device, dtype=F16)
    ldb = ldh = ldq = 0
    kb = None
    if key_bias is not None:
        kb = key_bias.to(device=q.device, dtype=torch.float32)
        if kb.dim() == 3:
            kb = kb.unsqueeze(2)
        if (kb.dim() != 4 or kb.shape[-1] != lk or kb.shape[0] not in (1, batch) or kb.shape[1] not in (1, heads)
                or kb.shape[2] not in (1, lq)):
            raise ValueError(f"key_bias must be [batch|1, heads|1, ({lq}|1,) {lk}], got {tuple(key_bias.shape)}")
        kb = kb.contiguous()
        ldb = kb.stride(0) if kb.shape[0] > 1 else 0
        ldh = kb.stride(1) if kb.shape[1] > 1 else 0
        ldq = kb.stride(2) if kb.shape[2] > 1 else 0
    C2D.attention_fwd(q, k, v, batch, heads, lq, lk, d, float(scale), kb, ldb, ldh, out, ldq)
    return out


def attention_small(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, batch: int, heads: int, l: int, d: int,
                    causal: bool, scale: float | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Short-sequence (l <= 128, d = 64) attention, optionally causal (c2d::attention_small)."""
    _require(q, "q")
    if scale is None:
        scale = 1.0 / math.sqrt(d)
    if out is None:
        out = torch.empty((batch * l, heads * d), device=q.device, dtype=F16)
    C2D.attention_small(q, k, v, batch, heads, l, d, float(scale), bool(causal), out)
    return out


def window_attention(qkv: torch.Tensor, row_map: torch.Tensor, n_windows: int, heads: int, d: int,
                     bias: torch.Tensor, mask: torch.Tensor | None, out: torch.Tensor) -> torch.Tensor:
    C2D.window_attention(qkv, row_map, n_windows, heads, d, bias, mask, out)
    return out


def htsat_mel_patches(mel: torch.Tensor, bn_scale: torch.Tensor, bn_shift: torch.Tensor) -> torch.Tensor:
    b, t, f = mel.shape
    assert f == 64 and mel.dtype == torch.float32 and mel.is_contiguous()
    out = torch.empty((b * 4096, 64), device=mel.device, dtype=F16)
    C2D.htsat_mel_patches(mel, bn_scale, bn_shift, out)
    return out


def patch_merge_gather(x: torch.Tensor, b: int, h: int, w: int, c: int) -> torch.Tensor:
    out = torch.empty((b * (h // 2) * (w // 2), 4 * c), device=x.device, dtype=F16)
    C2D.patch_merge_gather(x, b, h, w, c, out)
    return out


def row_mean(x: torch.Tensor, b: int, rows: int) -> torch.Tensor:
    out = torch.empty((b, x.shape[1]), device=x.device, dtype=torch.float32)
    C2D.row_mean(x, b, rows, out)
    return out


def softmax_rows(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Row softmax of a 2-D fp16 matrix (c2d::softmax_rows); out may alias x."""
    _require(x, "x")
    assert x.dim() == 2 and x.dtype == F16 and x.stride(1) == 1
    out = torch.empty_like(x) if out is None else out
    assert out.shape == x.shape and out.stride(1) == 1
    C2D.softmax_rows(x, out)
    return out


def l2_normalize_(x: torch.Tensor) -> torch.Tensor:
    C2D.l2_normalize(x)
    return x


def timestep_embedding(t_table: torch.Tensor, step_index: torch.Tensor | None, n: int, dim: int) -> torch.Tensor:
    out = torch.empty((n, dim), device=t_table.device, dtype=F16)
    C2D.timestep_embedding(t_table, step_index, n, dim, out)
    return out


def cfg_ddim_step(eps: torch.Tensor, x: torch.Tensor, guidance: float, coef: torch.Tensor, step_index: torch.Tensor,
                  advance: bool = True) -> torch.Tensor:
    C2D.cfg_ddim_step(eps, x, float(guidance), coef, step_index, bool(advance))
    return x


def latent_to_nhwc(x: torch.Tensor, cpad: int, dup: bool) -> torch.Tensor:
    b, c, hgt, wid = x.shape
    out = torch.empty(((2 if dup else 1) * b, hgt, wid, cpad), device=x.device, dtype=F16)
    C2D.latent_to_nhwc(x, cpad, bool(dup), out)
    return out


def upsample_nearest2x(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """NHWC fp16 nearest x2 (diffusers Upsample2D interpolate step)."""
    n, h, w, c = x.shape
    x = x.contiguous()
    if out is None:
        out = torch.empty(n, 2 * h, 2 * w, c, device=x.device, dtype=x.dtype)
    C2D.upsample_nearest2x(x, out)
    return out


def add(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    if out is None:
        out = torch.empty_like(a)
    C2D.add(a, b, out)
    return out
