"""The C-ABI library loads and exports every entry point include/c2d.h declares
(no compute calls: this runs on CPU-only machines)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "c2d.h").read_text()
    return sorted(set(re.findall(r"\b(c2d_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_core_entry_points():
    syms = declared_symbols()
    for s in ("c2d_conv2d_igemm", "c2d_groupnorm_stats", "c2d_attention_fwd", "c2d_window_attention",
              "c2d_cfg_ddim_step", "c2d_htsat_mel_patches"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import torch  # noqa: F401  (binds the library to torch's HIP runtime first)
    from clap2diffusion_amd import _lib
    if not _lib.LIB_PATH.exists():
        pytest.fail("libc2d_hip.so not built: run `python -m clap2diffusion_amd.build` (or __graft_entry__.build())")
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(_lib.EXPORTS) == set(declared_symbols())


def test_error_codes_without_gpu():
    """Argument validation happens before any HIP call."""
    import torch  # noqa: F401
    from clap2diffusion_amd import _lib
    L = _lib.lib()
    d = _lib.ConvDesc()
    assert L.c2d_conv2d_igemm(ctypes.byref(d), None) == -1   # null pointers -> C2D_E_ARG
    assert L.c2d_attention_fwd(None, 0, None, 0, None, 0, None, 0, 1, 1, 1, 1, 40, 1.0, 1, None) == -1
    d = _lib.ConvDesc()   # L3 (8x8) resnet conv at N=16: under-filled -> split-K workspace
    d.c0, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride, d.cout, d.kpad = 1280, 16, 8, 8, 8, 8, 3, 1, 1280, 11520
    assert L.c2d_conv2d_igemm_workspace_size(ctypes.byref(d)) % (16 * 64 * 1280 * 4) == 0
    assert L.c2d_conv2d_igemm_workspace_size(ctypes.byref(d)) >= 2 * 16 * 64 * 1280 * 4
    d.c0, d.h, d.w, d.oh, d.ow, d.cout, d.kpad = 320, 64, 64, 64, 64, 320, 2880   # L0: fills the chip
    assert L.c2d_conv2d_igemm_workspace_size(ctypes.byref(d)) == 0
    ws = L.c2d_groupnorm_workspace_size(2, 320, 4096)   # n * nblk * c * (sum, sumsq) fp32
    assert ws > 0 and ws % (2 * 320 * 2 * 4) == 0 and ws // (2 * 320 * 2 * 4) <= 4096
    assert L.c2d_version().startswith(b"c2d_hip gfx950")


def test_new_entry_points_validate_before_launch():
    """log-mel / short attention / row softmax: documented C2D_E_* codes, nothing launched."""
    import torch  # noqa: F401
    from clap2diffusion_amd import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(64)            # host memory: never dereferenced on these paths
    p = ctypes.cast(buf, ctypes.c_void_p)
    # c2d_clap_log_mel: null -> ARG; n_fft != 1024 or max_len <= n_fft/2 -> SHAPE; b == 0 -> OK
    assert L.c2d_clap_log_mel(None, p, p, 1, 480000, 1024, 480, p, p, p, 64, p, None) == -1
    assert L.c2d_clap_log_mel(p, p, p, 1, 480000, 2048, 480, p, p, p, 64, p, None) == -2
    assert L.c2d_clap_log_mel(p, p, p, 1, 400, 1024, 480, p, p, p, 64, p, None) == -2
    assert L.c2d_clap_log_mel(p, p, p, 0, 480000, 1024, 480, p, p, p, 64, p, None) == 0
    # c2d_attention_small: d != 64 or l > 128 -> SHAPE; batch 0 -> OK
    assert L.c2d_attention_small(p, 192, p, 192, p, 192, p, 64, 1, 1, 77, 40, 0.125, 1, None) == -2
    assert L.c2d_attention_small(p, 192, p, 192, p, 192, p, 64, 1, 1, 129, 64, 0.125, 1, None) == -2
    assert L.c2d_attention_small(None, 192, p, 192, p, 192, p, 64, 1, 1, 77, 64, 0.125, 1, None) == -1
    assert L.c2d_attention_small(p, 192, p, 192, p, 192, p, 64, 0, 1, 77, 64, 0.125, 1, None) == 0
    # c2d_softmax_rows: cols % 8, cols > 16384 -> SHAPE; misaligned ld -> ALIGN; rows 0 -> OK
    aligned = ctypes.c_void_p((ctypes.addressof(buf) + 15) & ~15)
    assert L.c2d_softmax_rows(aligned, 4, 12, 16, aligned, 16, None) == -2
    assert L.c2d_softmax_rows(aligned, 4, 16392, 16392, aligned, 16392, None) == -2
    assert L.c2d_softmax_rows(aligned, 4, 16, 20, aligned, 16, None) == -3
    assert L.c2d_softmax_rows(aligned, 0, 16, 16, aligned, 16, None) == 0
