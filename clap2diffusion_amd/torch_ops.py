"""torch.library custom ops over the C ABI ("callers via torch.library
custom-op wrappers that pass torch.cuda.current_stream()").

Every entry point of include/c2d.h that the sampling path calls is registered as a
``c2d::<name>`` operator with a CUDA (HIP) implementation only -- a CPU tensor reaching one
fails in the dispatcher, there is no fallback -- and a fake (meta) implementation, so the
ops are visible to torch (FakeTensor tracing, torch.compile graphs, schema checks) rather
than opaque ctypes calls.  All ops are out-variants: the caller (clap2diffusion_amd.ops)
allocates the outputs, the op mutates them (``mutates_args``) and returns nothing, which
keeps the fake implementations trivial and lets a GEMM write its result into the
residual it adds (in-place residual epilogues).  Each launch goes to
torch.cuda.current_stream(), so the ops are hipGraph-capturable as they stand.
"""
import ctypes
from typing import Optional

import torch
from torch import Tensor
from torch.library import custom_op

from ._lib import C2D_PRO_GN, C2D_PRO_LN, C2D_PRO_LNFOLD, C2D_PRO_NONE, C2D_PRO_SILU, ConvDesc, check, lib, ptr, stream_ptr

_CU = "cuda"


def _conv_desc(x, weight, kpad, cout, ksize, stride, up, x2, gn_scale, gn_shift, gn_silu, ln_stats, ln_gamma,
               ln_beta, silu_in, bias, act, temb, resid, out, src_pad=False, lnf_eps=0.0, gn_mom=None,
               gn_groups=0) -> ConvDesc:
    if x.dim() == 2:
        n, h, w = 1, 1, x.shape[0]
        c0 = x.shape[1]
    else:
        n, h, w, c0 = x.shape
        if src_pad:   # zero-bordered [n][h + 2][w + 2][c0]: logical size h x w
            h, w = h - 2, w - 2
    c1 = x2.shape[-1] if x2 is not None else 0
    if ksize == 3:
        vh, vw = (2 * h, 2 * w) if up else (h, w)
        oh, ow = (vh + 2 - 3) // stride + 1, (vw + 2 - 3) // stride + 1
    else:
        oh, ow = h, w
    d = ConvDesc()
    d.src0 = ptr(x); d.src1 = ptr(x2); d.c0 = c0; d.c1 = c1
    d.n, d.h, d.w, d.oh, d.ow = n, h, w, oh, ow
    d.ksize, d.stride, d.up = ksize, stride, int(up)
    d.weight = ptr(weight); d.cout = cout; d.kpad = kpad
    if lnf_eps > 0.0:   # LayerNorm folded into the panel GEMM (weight = W diag(gamma), bias = b + W beta)
        d.pro = C2D_PRO_LNFOLD; d.pro_eps = lnf_eps
    elif gn_scale is not None:
        d.pro = C2D_PRO_GN; d.pro_silu = int(gn_silu); d.pro_a = ptr(gn_scale); d.pro_b = ptr(gn_shift)
    elif ln_stats is not None:
        d.pro = C2D_PRO_LN; d.pro_a = ptr(ln_stats); d.gamma = ptr(ln_gamma); d.beta = ptr(ln_beta)
    elif silu_in:
        d.pro = C2D_PRO_SILU
    else:
        d.pro = C2D_PRO_NONE
    d.bias = ptr(bias)
    d.act = act
    if temb is not None:
        d.temb = ptr(temb); d.temb_ld = temb.stride(0)
    if resid is not None:
        d.resid = ptr(resid); d.resid_ld = resid.stride(-2) if resid.dim() == 2 else resid.shape[-1]
    d.out = ptr(out)
    d.out_ld = out.stride(-2) if out.dim() == 2 else out.shape[-1]
    d.src_pad = int(src_pad)
    if gn_mom is not None:
        d.gn_mom = ptr(gn_mom); d.gn_groups = gn_groups
    return d


_plan_probe: Optional[list] = None


@custom_op("c2d::conv2d_igemm", mutates_args=("out",), device_types=_CU)
def conv2d_igemm(x: Tensor, weight: Tensor, kpad: int, cout: int, ksize: int, stride: int, up: bool,
                 x2: Optional[Tensor], gn_scale: Optional[Tensor], gn_shift: Optional[Tensor], gn_silu: bool,
                 ln_stats: Optional[Tensor], ln_gamma: Optional[Tensor], ln_beta: Optional[Tensor], silu_in: bool,
                 bias: Optional[Tensor], act: int, temb: Optional[Tensor], resid: Optional[Tensor],
                 out: Tensor, src_pad: bool = False, lnf_eps: float = 0.0, gn_mom: Optional[Tensor] = None,
                 gn_groups: int = 0) -> None:
    """c2d_conv2d_igemm (+ its split-K workspace, sized by c2d_conv2d_igemm_workspace_size).
    src_pad: x is the zero-bordered layout [n][h + 2][w + 2][c] (c2d_groupnorm_pad).
    lnf_eps > 0: a LayerNorm (that eps) folded into the GEMM (C2D_PRO_LNFOLD).
    gn_mom: fp32 [n][hw / rows][gn_groups][2], the output's GroupNorm moments written by the conv
    (c2d_conv_desc::gn_mom; rows = c2d_conv2d_gn_rows)."""
    d = _conv_desc(x, weight, kpad, cout, ksize, stride, up, x2, gn_scale, gn_shift, gn_silu, ln_stats, ln_gamma,
                   ln_beta, silu_in, bias, act, temb, resid, out, src_pad, lnf_eps, gn_mom, gn_groups)
    wsb = lib().c2d_conv2d_igemm_workspace_size(ctypes.byref(d))
    if wsb:
        ws = torch.empty(wsb // 4, device=x.device, dtype=torch.float32)
        d.ws = ptr(ws); d.ws_bytes = wsb
    if _plan_probe is not None:
        tid, ks = ctypes.c_int(), ctypes.c_int()
        check(lib().c2d_conv2d_igemm_plan(ctypes.byref(d), ctypes.byref(tid), ctypes.byref(ks)), "c2d_conv2d_igemm_plan")
        _plan_probe.append((tid.value, ks.value))
    check(lib().c2d_conv2d_igemm(ctypes.byref(d), stream_ptr()), "c2d_conv2d_igemm")


@conv2d_igemm.register_fake
def _(x, weight, kpad, cout, ksize, stride, up, x2, gn_scale, gn_shift, gn_silu, ln_stats, ln_gamma, ln_beta,
      silu_in, bias, act, temb, resid, out, src_pad=False, lnf_eps=0.0, gn_mom=None, gn_groups=0):
    return None


@custom_op("c2d::pack_weights", mutates_args=("out",), device_types=_CU)
def pack_weights(w: Tensor, cout: int, cin: int, ksize: int, cin_pad: int, kpad: int, out: Tensor) -> None:
    check(lib().c2d_pack_weights(ptr(w), cout, cin, ksize, cin_pad, kpad, ptr(out), stream_ptr()), "c2d_pack_weights")


@custom_op("c2d::groupnorm_stats", mutates_args=("scale", "shift"), device_types=_CU)
def groupnorm_stats(x: Tensor, x2: Optional[Tensor], groups: int, eps: float, gamma: Tensor, beta: Tensor,
                    scale: Tensor, shift: Tensor) -> None:
    n, c0 = x.shape[0], x.shape[-1]
    c1 = x2.shape[-1] if x2 is not None else 0
    hw = x.numel() // (n * c0)
    ws = torch.empty(lib().c2d_groupnorm_workspace_size(n, c0 + c1, hw) // 4, device=x.device, dtype=torch.float32)
    check(lib().c2d_groupnorm_stats(ptr(x), ptr(x2), c0, c1, n, hw, groups, eps, ptr(gamma), ptr(beta), ptr(scale),
                                    ptr(shift), ptr(ws), stream_ptr()), "c2d_groupnorm_stats")


@custom_op("c2d::groupnorm_apply", mutates_args=("out",), device_types=_CU)
def groupnorm_apply(x: Tensor, x2: Optional[Tensor], scale: Tensor, shift: Tensor, silu: bool, out: Tensor) -> None:
    n, c0 = x.shape[0], x.shape[-1]
    c1 = x2.shape[-1] if x2 is not None else 0
    hw = x.numel() // (n * c0)
    check(lib().c2d_groupnorm_apply(ptr(x), ptr(x2), c0, c1, n, hw, ptr(scale), ptr(shift), int(silu), ptr(out),
                                    stream_ptr()), "c2d_groupnorm_apply")


@custom_op("c2d::groupnorm", mutates_args=("out",), device_types=_CU)
def groupnorm(x: Tensor, x2: Optional[Tensor], groups: int, eps: float, gamma: Tensor, beta: Tensor, silu: bool,
              out: Tensor) -> None:
    n, c0 = x.shape[0], x.shape[-1]
    c1 = x2.shape[-1] if x2 is not None else 0
    hw = x.numel() // (n * c0)
    wsb = lib().c2d_groupnorm_run_workspace_size(n, c0 + c1, hw, groups)
    ws = torch.empty((wsb + 15) // 16 * 4, device=x.device, dtype=torch.float32) if wsb else None
    check(lib().c2d_groupnorm(ptr(x), ptr(x2), c0, c1, n, hw, groups, eps, ptr(gamma), ptr(beta), int(silu), ptr(out),
                              ptr(ws), wsb, stream_ptr()), "c2d_groupnorm")


@custom_op("c2d::groupnorm_pad", mutates_args=("out",), device_types=_CU)
def groupnorm_pad(x: Tensor, x2: Optional[Tensor], groups: int, eps: float, gamma: Tensor, beta: Tensor, silu: bool,
                  out: Tensor) -> None:
    """c2d_groupnorm_pad: x [n][h][w][c0] (+ x2) -> out [n][h + 2][w + 2][c0 + c1], zero border."""
    n, h, w, c0 = x.shape
    c1 = x2.shape[-1] if x2 is not None else 0
    wsb = lib().c2d_groupnorm_pad_workspace_size(n, c0 + c1, h, w)
    ws = torch.empty((wsb + 15) // 16 * 4, device=x.device, dtype=torch.float32)
    check(lib().c2d_groupnorm_pad(ptr(x), ptr(x2), c0, c1, n, h, w, groups, eps, ptr(gamma), ptr(beta), int(silu),
                                  ptr(out), ptr(ws), wsb, stream_ptr()), "c2d_groupnorm_pad")


@custom_op("c2d::groupnorm_moments", mutates_args=("out",), device_types=_CU)
def groupnorm_moments(x: Tensor, groups: int, eps: float, gamma: Tensor, beta: Tensor, silu: bool, mom: Tensor,
                      rows: int, pad: bool, out: Tensor) -> None:
    """c2d_groupnorm_moments: x [n][h][w][c] normalised with the {mean, M2} moments its producing conv
    wrote (mom [n][h*w / rows][groups][2]) -> out [n][h][w][c], or with pad the zero-bordered
    [n][h + 2][w + 2][c]."""
    n, h, w, c = x.shape
    check(lib().c2d_groupnorm_moments(ptr(x), c, n, h * w, groups, eps, ptr(gamma), ptr(beta), int(silu), ptr(mom),
                                      rows, w + 2 if pad else 0, ptr(out), stream_ptr()), "c2d_groupnorm_moments")


@custom_op("c2d::layernorm_stats", mutates_args=("stats",), device_types=_CU)
def layernorm_stats(x: Tensor, eps: float, stats: Tensor) -> None:
    m, c = x.shape
    check(lib().c2d_layernorm_stats(ptr(x), m, c, x.stride(0), eps, ptr(stats), stream_ptr()), "c2d_layernorm_stats")


@custom_op("c2d::layernorm", mutates_args=("out",), device_types=_CU)
def layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float, out: Tensor) -> None:
    m, c = x.shape
    check(lib().c2d_layernorm(ptr(x), m, c, x.stride(0), eps, ptr(gamma), ptr(beta), ptr(out), out.stride(0),
                              stream_ptr()), "c2d_layernorm")


@custom_op("c2d::attention_fwd", mutates_args=("out",), device_types=_CU)
def attention_fwd(q: Tensor, k: Tensor, v: Tensor, batch: int, heads: int, lq: int, lk: int, d: int, scale: float,
                  key_bias: Optional[Tensor], bias_ld_batch: int, bias_ld_head: int, out: Tensor,
                  bias_ld_query: int = 0) -> None:
    """c2d_attention_fwd, or c2d_attention_fwd_mask with an additive score bias (bias_ld_query 0:
    a per-key bias, else a query-varying one)."""
    if key_bias is None:
        check(lib().c2d_attention_fwd(ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
                                      out.stride(0), batch, heads, lq, lk, d, scale, 1, stream_ptr()), "c2d_attention_fwd")
    else:
        check(lib().c2d_attention_fwd_mask(ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
                                           out.stride(0), batch, heads, lq, lk, d, scale, 1, ptr(key_bias),
                                           bias_ld_batch, bias_ld_head, bias_ld_query, stream_ptr()),
              "c2d_attention_fwd_mask")


@custom_op("c2d::attention_small", mutates_args=("out",), device_types=_CU)
def attention_small(q: Tensor, k: Tensor, v: Tensor, batch: int, heads: int, l: int, d: int, scale: float,
                    causal: bool, out: Tensor) -> None:
    check(lib().c2d_attention_small(ptr(q), q.stride(0), ptr(k), k.stride(0), ptr(v), v.stride(0), ptr(out),
                                    out.stride(0), batch, heads, l, d, scale, int(causal), stream_ptr()),
          "c2d_attention_small")


@custom_op("c2d::window_attention", mutates_args=("out",), device_types=_CU)
def window_attention(qkv: Tensor, row_map: Tensor, n_windows: int, heads: int, d: int, bias: Tensor,
                     mask: Optional[Tensor], out: Tensor) -> None:
    n_mask = mask.shape[0] if mask is not None else 0
    check(lib().c2d_window_attention(ptr(qkv), qkv.stride(0), ptr(row_map), n_windows, heads, d, ptr(bias), ptr(mask),
                                     n_mask, ptr(out), out.stride(0), stream_ptr()), "c2d_window_attention")


@custom_op("c2d::htsat_mel_patches", mutates_args=("out",), device_types=_CU)
def htsat_mel_patches(mel: Tensor, bn_scale: Tensor, bn_shift: Tensor, out: Tensor) -> None:
    b, t, _ = mel.shape
    check(lib().c2d_htsat_mel_patches(ptr(mel), b, t, ptr(bn_scale), ptr(bn_shift), ptr(out), stream_ptr()),
          "c2d_htsat_mel_patches")


@custom_op("c2d::patch_merge_gather", mutates_args=("out",), device_types=_CU)
def patch_merge_gather(x: Tensor, b: int, h: int, w: int, c: int, out: Tensor) -> None:
    check(lib().c2d_patch_merge_gather(ptr(x), b, h, w, c, ptr(out), stream_ptr()), "c2d_patch_merge_gather")


@custom_op("c2d::row_mean", mutates_args=("out",), device_types=_CU)
def row_mean(x: Tensor, b: int, rows: int, out: Tensor) -> None:
    check(lib().c2d_row_mean(ptr(x), b, rows, x.shape[1], x.stride(0), ptr(out), stream_ptr()), "c2d_row_mean")


@custom_op("c2d::softmax_rows", mutates_args=("out",), device_types=_CU)
def softmax_rows(x: Tensor, out: Tensor) -> None:
    check(lib().c2d_softmax_rows(ptr(x), x.shape[0], x.shape[1], x.stride(0), ptr(out), out.stride(0), stream_ptr()),
          "c2d_softmax_rows")


@custom_op("c2d::l2_normalize", mutates_args=("x",), device_types=_CU)
def l2_normalize(x: Tensor) -> None:
    m, c = x.shape
    check(lib().c2d_l2_normalize(ptr(x), m, c, stream_ptr()), "c2d_l2_normalize")


@custom_op("c2d::clap_log_mel", mutates_args=("out",), device_types=_CU)
def clap_log_mel(wave: Tensor, offsets: Tensor, lengths: Tensor, max_len: int, n_fft: int, hop: int, window: Tensor,
                 filters: Tensor, filter_range: Tensor, n_mels: int, out: Tensor) -> None:
    check(lib().c2d_clap_log_mel(ptr(wave), ptr(offsets), ptr(lengths), offsets.numel(), max_len, n_fft, hop,
                                 ptr(window), ptr(filters), ptr(filter_range), n_mels, ptr(out), stream_ptr()),
          "c2d_clap_log_mel")


@custom_op("c2d::timestep_embedding", mutates_args=("out",), device_types=_CU)
def timestep_embedding(t_table: Tensor, step_index: Optional[Tensor], n: int, dim: int, out: Tensor) -> None:
    check(lib().c2d_timestep_embedding(ptr(t_table), ptr(step_index), n, dim, ptr(out), stream_ptr()),
          "c2d_timestep_embedding")


@custom_op("c2d::cfg_ddim_step", mutates_args=("x", "step_index"), device_types=_CU)
def cfg_ddim_step(eps: Tensor, x: Tensor, guidance: float, coef: Tensor, step_index: Tensor, advance: bool) -> None:
    b, c, hgt, wid = x.shape
    check(lib().c2d_cfg_ddim_step(ptr(eps), ptr(x), b, c, hgt * wid, guidance, ptr(coef), ptr(step_index), int(advance),
                                  stream_ptr()), "c2d_cfg_ddim_step")


@custom_op("c2d::latent_to_nhwc", mutates_args=("out",), device_types=_CU)
def latent_to_nhwc(x: Tensor, cpad: int, dup: bool, out: Tensor) -> None:
    b, c, hgt, wid = x.shape
    check(lib().c2d_latent_to_nhwc(ptr(x), b, c, hgt * wid, cpad, int(dup), ptr(out), stream_ptr()),
          "c2d_latent_to_nhwc")


@custom_op("c2d::upsample_nearest2x", mutates_args=("out",), device_types=_CU)
def upsample_nearest2x(x: Tensor, out: Tensor) -> None:
    n, h, w, c = x.shape
    check(lib().c2d_upsample_nearest2x(ptr(x), n, h, w, c, ptr(out), stream_ptr()), "c2d_upsample_nearest2x")


@custom_op("c2d::add", mutates_args=("out",), device_types=_CU)
def add(a: Tensor, b: Tensor, out: Tensor) -> None:
    check(lib().c2d_add(ptr(a), ptr(b), ptr(out), a.numel(), stream_ptr()), "c2d_add")


# fake (meta) implementations: every op only mutates caller-allocated outputs
for _op in (pack_weights, groupnorm_stats, groupnorm_apply, groupnorm, groupnorm_pad, groupnorm_moments, layernorm_stats, layernorm, attention_fwd,
            attention_small, window_attention, htsat_mel_patches, patch_merge_gather, row_mean, softmax_rows,
            l2_normalize, clap_log_mel, timestep_embedding, cfg_ddim_step, latent_to_nhwc, upsample_nearest2x, add):
    _op.register_fake(lambda *args, **kwargs: None)

OPS = ("conv2d_igemm", "pack_weights", "groupnorm_stats", "groupnorm_apply", "groupnorm", "groupnorm_pad", "groupnorm_moments",
       "layernorm_stats",
       "layernorm", "attention_fwd", "attention_small", "window_attention", "htsat_mel_patches", "patch_merge_gather",
       "row_mean", "softmax_rows", "l2_normalize", "clap_log_mel", "timestep_embedding", "cfg_ddim_step",
       "latent_to_nhwc", "upsample_nearest2x", "add")
