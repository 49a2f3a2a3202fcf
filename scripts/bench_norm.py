"""Per-shape timing of GroupNorm stats (+ finalize) and apply on the UNet's norm shapes (N = 16)."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")
N = 16
SHAPES = [(64, 320, 0), (64, 640, 320), (32, 640, 0), (32, 1280, 640), (16, 1280, 0), (16, 1280, 1280),
          (8, 1280, 0), (8, 1280, 1280)]


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for h, c0, c1 in SHAPES:
    x = torch.randn(N, h, h, c0, device=dev, dtype=torch.float16) * 2 + 0.5
    x2 = torch.randn(N, h, h, c1, device=dev, dtype=torch.float16) if c1 else None
    c = c0 + c1
    g = torch.rand(c, device=dev) + 0.5
    b = torch.randn(c, device=dev) * 0.1
    st = lambda: ops.group_norm_stats(x, 32, 1e-5, g, b, x2=x2)  # noqa: E731
    t_st = timed(st)
    gn = st()
    out = torch.empty(N, h, h, c, device=dev, dtype=torch.float16)
    t_ap = timed(lambda: ops.group_norm_apply(x, gn, True, x2=x2, out=out))
    t_one = timed(lambda: ops.group_norm(x, 32, 1e-5, g, b, True, x2=x2, out=out))
    xc = torch.cat([x, x2], -1) if x2 is not None else x
    ref = F.silu(F.group_norm(xc.permute(0, 3, 1, 2).float(), 32, g, b, 1e-5)).permute(0, 2, 3, 1)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    mb = N * h * h * c * 2 / 1e6
    print(f"GN {h:3d}^2 c={c0}+{c1}: stats {t_st:7.1f} us ({mb / t_st:6.0f} GB/s)  apply {t_ap:7.1f} us "
          f"({2 * mb / t_ap:6.0f} GB/s)  one-call {t_one:7.1f} us  relerr {err:.1e}", flush=True)
