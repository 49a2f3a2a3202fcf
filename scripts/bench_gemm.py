"""Per-shape timing of c2d_conv2d_igemm on the UNet's hot conv/GEMM shapes (N = 16)."""
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ops.plan_override_from_env()   # C2D_GEMM_TILE / C2D_GEMM_SPLIT (tuning runs only)

dev = torch.device("cuda")
N = 16
SHAPES = [  # (name, ksize, h, cin, cout, M-rows for linear)
    ("L0 k64 64->320", 1, 64, 64, 320),
    ("L0 conv3x3 320", 3, 64, 320, 320),
    ("L1 conv3x3 640", 3, 32, 640, 640),
    ("L2 conv3x3 1280", 3, 16, 1280, 1280),
    ("L3 conv3x3 1280", 3, 8, 1280, 1280),
    ("L0 up conv3x3 960->320", 3, 64, 960, 320),
    ("L0 geglu 320->2560", 1, 64, 320, 2560),
    ("L0 ff2 1280->320", 1, 64, 1280, 320),
    ("L0 qkv 320->960", 1, 64, 320, 960),
    ("L0 proj 320->320", 1, 64, 320, 320),
    ("L1 geglu 640->5120", 1, 32, 640, 5120),
    ("L2 geglu 1280->10240", 1, 16, 1280, 10240),
    ("L1 ff2 2560->640", 1, 32, 2560, 640),
    ("L1 qkv 640->1920", 1, 32, 640, 1920),
    ("L2 conv 2560->1280", 3, 16, 2560, 1280),
    ("L1 up conv 1920->640", 3, 32, 1920, 640),
    ("L3 conv 2560->1280", 3, 8, 2560, 1280),
    ("L2 qkv 1280->3840", 1, 16, 1280, 3840),
    ("L1 proj 640->640", 1, 32, 640, 640),
    ("L2 proj 1280->1280", 1, 16, 1280, 1280),
    ("L2 ff2 5120->1280", 1, 16, 5120, 1280),
    ("L0 GEGLU act 320->2x1280", 1, 64, 320, 2560, "geglu"),
    ("VAE 512^2 conv 128->128 n2", 3, 512, 128, 128, None, 2),
    ("VAE 256^2 conv 256->256 n2", 3, 256, 256, 256, None, 2),
    ("VAE 512^2 conv 256->256 n2", 3, 512, 256, 256, None, 2),
    ("VAE 128^2 conv 512->512 n2", 3, 128, 512, 512, None, 2),
    ("VAE 64^2 conv 512->512 n8", 3, 64, 512, 512, None, 8),
    ("L1 GEGLU act 640->2x2560", 1, 32, 640, 5120, "geglu"),
]


def lib_gemm_us(m, kk, nn, iters=20):
    """hipBLASLt (torch.mm) time of the equivalent plain GEMM [m, kk] x [kk, nn] fp16 -- the
    im2col-free library ceiling for the same MACs (no conv addressing, no epilogue)."""
    a = torch.randn(m, kk, device=dev, dtype=torch.float16)
    b = torch.randn(kk, nn, device=dev, dtype=torch.float16)
    for _ in range(3):
        torch.mm(a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.mm(a, b)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def run(name, k, h, cin, cout, act=None, n=N, iters=20):
    x = torch.randn(n, h, h, cin, device=dev, dtype=torch.float16)
    w = torch.randn(cout, cin, k, k, device=dev) / math.sqrt(k * k * cin)
    wp, kp = ops.pack_conv_weight(w)
    out = torch.empty(n, h, h, cout // 2 if act == "geglu" else cout, device=dev, dtype=torch.float16)
    for _ in range(3):
        ops.conv(x, wp, kp, cout, ksize=k, out=out, act=act)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.conv(x, wp, kp, cout, ksize=k, out=out, act=act)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    fl = 2.0 * n * h * h * cout * k * k * cin
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w, padding=k // 2).permute(0, 2, 3, 1)
    if act == "geglu":   # packed [16 h | 16 g] column blocks (ops.geglu_interleave layout)
        r = ref.reshape(*ref.shape[:-1], -1, 2, 16)
        ref = (r[..., 0, :] * torch.nn.functional.gelu(r[..., 1, :])).reshape(*ref.shape[:-1], -1)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    hbm = 2.0 * (n * h * h * (cin + (cout // 2 if act == "geglu" else cout)) + cout * k * k * cin) / 5.0e6  # us at 5 TB/s
    lib = lib_gemm_us(n * h * h, k * k * cin, cout) if os.environ.get("LIB", "1") == "1" else float("nan")
    print(f"{name:26s} {ms * 1e3:9.1f} us {fl / ms / 1e9:8.1f} TF/s  hbm-floor {hbm:7.1f} us  hipblaslt-gemm {lib:7.1f} us "
          f"({fl / lib / 1e6:7.1f} TF/s)  relerr {err:.1e}", flush=True)


import os
only = os.environ.get("ONLY")
for s in SHAPES:
    if only and not any(o in s[0] for o in only.split(",")):
        continue
    run(*s)
