"""ctypes binding of libc2d_hip.so (include/c2d.h).

The library is the only compute path: importing this module on a machine
without the built library, or calling an op without a GPU, raises — there is
no CPU / PyTorch fallback behind these entry points.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_size_t, c_void_p
from pathlib import Path

import torch  # noqa: F401  (must be loaded first: the library binds to torch's libamdhip64.so.7)

LIB_PATH = Path(os.environ.get("C2D_LIB") or Path(__file__).resolve().parent / "libc2d_hip.so")  # C2D_LIB: A/B builds

C2D_PRO_NONE, C2D_PRO_GN, C2D_PRO_LN, C2D_PRO_SILU, C2D_PRO_LNFOLD = 0, 1, 2, 3, 4
C2D_ACT = {None: 0, "none": 0, "geglu": 1, "gelu": 2, "relu": 3, "silu": 4, "quick_gelu": 5}
ERRORS = {-1: "C2D_E_ARG", -2: "C2D_E_SHAPE", -3: "C2D_E_ALIGN", -4: "C2D_E_HIP"}

# every symbol include/c2d.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "c2d_conv2d_igemm", "c2d_conv2d_igemm_workspace_size", "c2d_conv2d_igemm_plan", "c2d_set_plan_override", "c2d_get_plan_override", "c2d_groupnorm_workspace_size", "c2d_groupnorm_stats", "c2d_groupnorm_apply", "c2d_groupnorm_run_workspace_size", "c2d_groupnorm", "c2d_groupnorm_pad_workspace_size", "c2d_groupnorm_pad", "c2d_conv2d_gn_rows", "c2d_groupnorm_moments", "c2d_layernorm_stats",
    "c2d_layernorm", "c2d_attention_fwd", "c2d_attention_fwd_bias", "c2d_attention_fwd_mask", "c2d_window_attention", "c2d_htsat_mel_patches",
    "c2d_patch_merge_gather", "c2d_row_mean", "c2d_l2_normalize", "c2d_softmax_rows", "c2d_clap_log_mel", "c2d_attention_small", "c2d_pack_weights", "c2d_timestep_embedding",
    "c2d_cfg_ddim_step", "c2d_latent_to_nhwc", "c2d_upsample_nearest2x", "c2d_add", "c2d_last_hip_error", "c2d_version",
]


class ConvDesc(ctypes.Structure):
    _fields_ = [
        ("src0", c_void_p), ("src1", c_void_p), ("c0", c_int), ("c1", c_int),
        ("n", c_int), ("h", c_int), ("w", c_int), ("oh", c_int), ("ow", c_int),
        ("ksize", c_int), ("stride", c_int), ("up", c_int),
        ("weight", c_void_p), ("cout", c_int), ("kpad", c_int),
        ("pro", c_int), ("pro_silu", c_int), ("pro_a", c_void_p), ("pro_b", c_void_p),
        ("gamma", c_void_p), ("beta", c_void_p), ("bias", c_void_p), ("act", c_int),
        ("temb", c_void_p), ("temb_ld", c_int), ("resid", c_void_p), ("resid_ld", c_int),
        ("out", c_void_p), ("out_ld", c_int), ("ws", c_void_p), ("ws_bytes", c_size_t),
        ("src_pad", c_int), ("pro_eps", c_float),
        ("gn_mom", c_void_p), ("gn_groups", c_int),   # r6: producer-emitted GroupNorm moments
    ]


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -m clap2diffusion_amd.build` "
            "(the HIP library is the only compute path; there is no fallback)")
    L = ctypes.CDLL(str(LIB_PATH))
    vp, i, f, sz = c_void_p, c_int, c_float, c_size_t
    sig = {
        "c2d_conv2d_igemm": ([ctypes.POINTER(ConvDesc), vp], i),
        "c2d_conv2d_igemm_workspace_size": ([ctypes.POINTER(ConvDesc)], sz),
        "c2d_conv2d_igemm_plan": ([ctypes.POINTER(ConvDesc), ctypes.POINTER(c_int), ctypes.POINTER(c_int)], i),
        "c2d_set_plan_override": ([i, i], i),
        "c2d_get_plan_override": ([ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], i),
        "c2d_groupnorm_workspace_size": ([i, i, i], sz),
        "c2d_groupnorm_stats": ([vp, vp, i, i, i, i, i, f, vp, vp, vp, vp, vp, vp], i),
        "c2d_groupnorm_apply": ([vp, vp, i, i, i, i, vp, vp, i, vp, vp], i),
        "c2d_groupnorm_run_workspace_size": ([i, i, i, i], sz),
        "c2d_groupnorm": ([vp, vp, i, i, i, i, i, f, vp, vp, i, vp, vp, sz, vp], i),
        "c2d_groupnorm_pad_workspace_size": ([i, i, i, i], sz),
        "c2d_groupnorm_pad": ([vp, vp, i, i, i, i, i, i, f, vp, vp, i, vp, vp, sz, vp], i),
        "c2d_conv2d_gn_rows": ([ctypes.POINTER(ConvDesc)], i),
        "c2d_groupnorm_moments": ([vp, i, i, i, i, f, vp, vp, i, vp, i, i, vp, vp], i),
        "c2d_layernorm_stats": ([vp, i, i, i, f, vp, vp], i),
        "c2d_layernorm": ([vp, i, i, i, f, vp, vp, vp, i, vp], i),
        "c2d_attention_fwd": ([vp, i, vp, i, vp, i, vp, i, i, i, i, i, i, f, i, vp], i),
        "c2d_attention_fwd_bias": ([vp, i, vp, i, vp, i, vp, i, i, i, i, i, i, f, i, vp, i, i, vp], i),
        "c2d_attention_fwd_mask": ([vp, i, vp, i, vp, i, vp, i, i, i, i, i, i, f, i, vp, i, i, i, vp], i),
        "c2d_window_attention": ([vp, i, vp, i, i, i, vp, vp, i, vp, i, vp], i),
        "c2d_htsat_mel_patches": ([vp, i, i, vp, vp, vp, vp], i),
        "c2d_patch_merge_gather": ([vp, i, i, i, i, vp, vp], i),
        "c2d_row_mean": ([vp, i, i, i, i, vp, vp], i),
        "c2d_l2_normalize": ([vp, i, i, vp], i),
        "c2d_softmax_rows": ([vp, i, i, i, vp, i, vp], i),
        "c2d_clap_log_mel": ([vp, vp, vp, i, i, i, i, vp, vp, vp, i, vp, vp], i),
        "c2d_attention_small": ([vp, i, vp, i, vp, i, vp, i, i, i, i, i, f, i, vp], i),
        "c2d_pack_weights": ([vp, i, i, i, i, i, vp, vp], i),
        "c2d_timestep_embedding": ([vp, vp, i, i, vp, vp], i),
        "c2d_cfg_ddim_step": ([vp, vp, i, i, i, f, vp, vp, i, vp], i),
        "c2d_latent_to_nhwc": ([vp, i, i, i, i, i, vp, vp], i),
        "c2d_upsample_nearest2x": ([vp, i, i, i, i, vp, vp], i),
        "c2d_add": ([vp, vp, vp, sz, vp], i),
        "c2d_last_hip_error": ([], i),
        "c2d_version": ([], ctypes.c_char_p),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        extra = ""
        if rc == -4:
            extra = f" (hipError {lib().c2d_last_hip_error()})"
        raise RuntimeError(f"{what} failed: {ERRORS.get(rc, rc)}{extra}")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def is_available() -> bool:
    return LIB_PATH.exists()


os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
