"""(tile, split-K) sweep of the under-filled UNet conv / GEMM shapes (N = 16), one process:
The plan is forced through c2d_set_plan_override (ops.force_plan).  Prints the default plan's time and the
best forced (tile, split) per shape.  python scripts/sweep_split.py"""
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")
N = 16
SHAPES = [  # name, ksize, h, cin, cout, resid
    ("L3 3x3 1280 +res", 3, 8, 1280, 1280, True),
    ("L3 3x3 2560->1280", 3, 8, 2560, 1280, False),
    ("L2 3x3 1280 +res", 3, 16, 1280, 1280, True),
    ("L2 3x3 2560->1280", 3, 16, 2560, 1280, False),
    ("L1 3x3 640 +res", 3, 32, 640, 640, True),
    ("L2 1x1 1280 +res", 1, 16, 1280, 1280, True),
    ("L2 1x1 5120->1280 +res", 1, 16, 5120, 1280, True),
    ("mid 1x1 1280 +res", 1, 8, 1280, 1280, True),
]
TILES = [7, 1, 2, 3, 40, 41]
SPLITS = [1, 2, 3, 4, 6, 8]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for name, k, h, cin, cout, res in SHAPES:
    x = torch.randn(N, h, h, cin, device=dev, dtype=torch.float16)
    w = torch.randn(cout, cin, k, k, device=dev) / math.sqrt(k * k * cin)
    b = torch.randn(cout, device=dev)
    r = torch.randn(N, h, h, cout, device=dev, dtype=torch.float16) if res else None
    wp, kp = ops.pack_conv_weight(w)
    out = torch.empty(N, h, h, cout, device=dev, dtype=torch.float16)
    fn = lambda: ops.conv(x, wp, kp, cout, ksize=k, bias=b, resid=r, out=out)  # noqa: E731
    ops.force_plan(0, 0).__enter__()
    with ops.record_conv_plans() as pl:
        fn()
    base = timeit(fn)
    ref = out.float().clone()
    res_t = []
    for t in TILES:
        for s in SPLITS:
            ops.force_plan(t, s).__enter__()
            with ops.record_conv_plans() as pl2:
                fn()
            if pl2[0] != (t, s):
                continue
            us = timeit(fn)
            err = ((out.float() - ref).norm() / ref.norm()).item()
            res_t.append((us, t, s, err))
    ops.force_plan(0, 0).__enter__()
    res_t.sort()
    best = " ".join(f"({t},{s}) {us:.1f}" for us, t, s, _ in res_t[:5])
    print(f"{name:26s} default {pl[0]} {base:7.1f} us | best: {best} | max relerr {max(e for *_, e in res_t):.1e}",
          flush=True)
