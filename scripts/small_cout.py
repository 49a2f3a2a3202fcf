"""Forced-tile timing of the narrow-output convs (UNet conv_out 320 -> 4 at 64^2, N = 16; VAE
post_quant / conv_out shapes): which tile the planner should give a cout << tile width."""
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")
for name, n, h, cin, cout in [("unet conv_out", 16, 64, 320, 4), ("vae conv_out", 8, 512, 128, 4),
                              ("conv_out 320->8", 16, 64, 320, 8)]:
    x = torch.randn(n, h, h, cin, device=dev, dtype=torch.float16)
    w = torch.randn(cout, cin, 3, 3, device=dev) / math.sqrt(9 * cin)
    b = torch.randn(cout, device=dev)
    wp, kp = ops.pack_conv_weight(w)
    out = torch.empty(n, h, h, cout, device=dev, dtype=torch.float16)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w, b, padding=1).permute(0, 2, 3, 1)
    for t in (0, 40, 7, 1, 2, 3, 29):
        if t:
            ops.force_plan(t, 0).__enter__()
        else:
            ops.force_plan(0, 0).__enter__()
        with ops.record_conv_plans() as pl:
            ops.conv(x, wp, kp, cout, ksize=3, bias=b, out=out)
        for _ in range(2):
            ops.conv(x, wp, kp, cout, ksize=3, bias=b, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.conv(x, wp, kp, cout, ksize=3, bias=b, out=out)
        e1.record()
        e1.synchronize()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        print(f"{name:16s} forced {t:2d} plan {pl[0]} {e0.elapsed_time(e1) / 10 * 1e3:8.1f} us  relerr {err:.1e}",
              flush=True)
    ops.force_plan(0, 0).__enter__()
