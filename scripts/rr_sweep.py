"""Row-ring split sweep: every stride-1 3x3 ResnetBlock2D conv shape of the UNet at a batch, the
production route (unpadded source, the planner's plan) against the row-ring tile of that width
(42 / 43 / 44) on the zero-bordered source with every K split of whole channel blocks.
Graph-replayed device time per call; prints the best row-ring plan per shape and a kRrHints line
where it wins by >= 3 %.   python scripts/rr_sweep.py --batch 1 [--iters 20]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402
from rowring_ab import timed  # noqa: E402  (graph-replayed timing)

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--only-h", type=int, default=0, help="only shapes at this latent side")
ap.add_argument("--prefix", action="store_true",
                help="the CFG-shared prefix's first ResnetBlock2D (N = batch, level 0, 320 -> 320)")
a = ap.parse_args()
dev = torch.device("cuda")
N = a.batch if a.prefix else 2 * a.batch
SHAPES = [  # h, cin, cout (conv1: +temb when cin != cout, conv2: +res)
    (64, 320, 320), (64, 640, 320), (64, 960, 320),
    (32, 320, 640), (32, 640, 640), (32, 960, 640), (32, 1280, 640), (32, 1920, 640),
    (16, 640, 1280), (16, 1280, 1280), (16, 1920, 1280), (16, 2560, 1280),
]
if a.prefix:
    SHAPES = [(64, 320, 320)]
RR = {64: (42,), 32: (43,), 16: (44,)}
g = torch.Generator().manual_seed(0)
for h, cin, cout in SHAPES:
    if a.only_h and h != a.only_h:
        continue
    x = (torch.randn(N, h, h, cin, generator=g)).half().to(dev)
    xp = torch.zeros(N, h + 2, h + 2, cin, dtype=torch.float16, device=dev)
    xp[:, 1:-1, 1:-1] = x
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(9 * cin)
    wp, kp = ops.pack_conv_weight(w)
    wp = wp.to(dev)
    b = torch.zeros(cout, device=dev)
    temb = torch.randn(N, cout, generator=g).half().to(dev) if cin != cout else None
    res = torch.randn(N, h, h, cout, generator=g).half().to(dev) if cin == cout else None
    out = torch.empty(N, h, h, cout, dtype=torch.float16, device=dev)
    with ops.record_conv_plans() as rec:
        ops.conv(x, wp, kp, cout, ksize=3, bias=b, temb=temb, resid=res, out=out)
    ref = out.clone()
    base = timed(lambda: ops.conv(x, wp, kp, cout, ksize=3, bias=b, temb=temb, resid=res, out=out), a.iters)
    ncb = cin // 64
    best = None
    for tid in RR[h]:
        for sp in sorted({s for s in (1, 2, 3, 4, 5, 6, 8, 10, 12, 15, 16, 20, 24, 30, 40) if s <= ncb}):
            with ops.force_plan(tid, sp):
                with ops.record_conv_plans() as r2:
                    ops.conv(xp, wp, kp, cout, ksize=3, bias=b, temb=temb, resid=res, out=out, padded=True)
                if r2[0] != (tid, sp):
                    continue
                err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                us = timed(lambda: ops.conv(xp, wp, kp, cout, ksize=3, bias=b, temb=temb, resid=res, out=out,
                                            padded=True), a.iters)
            print(f"  N={N} {h}^2 {cin}->{cout}: ({tid}, {sp}) {us:7.1f} us  (vs production {base:.1f}, diff {err:.1e})",
                  flush=True)
            if best is None or us < best[2]:
                best = (tid, sp, us)
    m = N * h * h
    tag = "WIN" if best and best[2] < 0.97 * base else "keep"
    print(f"{tag} N={N} {h}^2 {cin}->{cout}: production {rec[0]} {base:.1f} us; best row ring ({best[0]}, {best[1]}) "
          f"{best[2]:.1f} us", flush=True)
    if tag == "WIN":
        print(f"    {{{m}, {9 * cin}, {cout}, {best[0]}, {best[1]}}},   // N = {N} {h}^2 {cin} -> {cout}: "
              f"{base:.1f} -> {best[2]:.1f} us", flush=True)
