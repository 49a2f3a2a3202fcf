"""(tile, split-K) sweep of UNet conv / GEMM shapes with graph-replayed timing.

Eager back-to-back launches of a kernel shorter than the host's per-call cost time the host,
not the device (the N = 2 shapes all read ~23 us that way); here `iters` calls are captured
in one hipGraph and replayed between HIP events, so the figure is device time per call.
python scripts/sweep_tiles_graph.py [--batch 8] [--only substr] [--tiles 40,41,...]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--only", default="")
ap.add_argument("--tiles", default="40,41,25,7,1,2,3,8,9")
ap.add_argument("--splits", default="1,2,3,4,6,8")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--res", type=int, default=64, help="latent side at level 0")
ap.add_argument("--vae", action="store_true", help="the VAE decoder's conv shapes (N = --batch)")
a = ap.parse_args()
dev = torch.device("cuda")
N = a.batch if a.vae else 2 * a.batch
SHAPES = [  # name, ksize, h (latent side at that level), cin, cout, resid, temb
    ("L0 1x1 320 +res", 1, 64, 320, 320, True, False),
    ("L0 1x1 320", 1, 64, 320, 320, False, False),
    ("L0 1x1 1280->320 +res", 1, 64, 1280, 320, True, False),
    ("L0 qkv 320->960", 1, 64, 320, 960, False, False),
    ("L1 1x1 640 +res", 1, 32, 640, 640, True, False),
    ("L1 1x1 640", 1, 32, 640, 640, False, False),
    ("L1 1x1 2560->640 +res", 1, 32, 2560, 640, True, False),
    ("L1 qkv 640->1920", 1, 32, 640, 1920, False, False),
    ("L2 1x1 1280 +res", 1, 16, 1280, 1280, True, False),
    ("L2 1x1 1280", 1, 16, 1280, 1280, False, False),
    ("L2 1x1 5120->1280 +res", 1, 16, 5120, 1280, True, False),
    ("L2 qkv 1280->3840", 1, 16, 1280, 3840, False, False),
    ("L3 1x1 1280 +res", 1, 8, 1280, 1280, True, False),
    ("L0 3x3 320 +res", 3, 64, 320, 320, True, False),
    ("L1 3x3 640 +res", 3, 32, 640, 640, True, False),
    ("L1 3x3 1920->640 +temb", 3, 32, 1920, 640, False, True),
    ("L2 3x3 1280 +res", 3, 16, 1280, 1280, True, False),
    ("L2 3x3 2560->1280 +temb", 3, 16, 2560, 1280, False, True),
    ("L3 3x3 1280 +res", 3, 8, 1280, 1280, True, False),
    ("L3 3x3 2560->1280 +temb", 3, 8, 2560, 1280, False, True),
    ("L0 3x3 640->320 +temb", 3, 64, 640, 320, False, True),
    ("L0 3x3 960->320 +temb", 3, 64, 960, 320, False, True),
    ("L1 3x3 1280->640 +temb", 3, 32, 1280, 640, False, True),
    ("L1 3x3 960->640 +temb", 3, 32, 960, 640, False, True),
    ("L2 3x3 1920->1280 +temb", 3, 16, 1920, 1280, False, True),
    ("L1 geglu 640->5120", 1, 32, 640, 5120, False, False),
    ("L2 geglu 1280->10240", 1, 16, 1280, 10240, False, False),
    ("L0 geglu 320->2560", 1, 64, 320, 2560, False, False),
    # ff.net.2 folded into proj_out: K = C (h) + 4C (GEGLU out, a second source), + residual
    ("L0 fold 320+1280->320 +res", 1, 64, 320, 320, True, False, 1280),
    ("L1 fold 640+2560->640 +res", 1, 32, 640, 640, True, False, 2560),
    ("L2 fold 1280+5120->1280 +res", 1, 16, 1280, 1280, True, False, 5120),
    ("L3 fold 1280+5120->1280 +res", 1, 8, 1280, 1280, True, False, 5120),
]
VAE_SHAPES = [  # AutoencoderKL decoder convs (SD1.5: 512 / 512 / 256 / 128 channels at 64 / 128 / 256 / 512^2)
    ("VAE 64^2 3x3 512 +res", 3, 64, 512, 512, True, False),
    ("VAE 128^2 3x3 512 +res", 3, 128, 512, 512, True, False),
    ("VAE 256^2 3x3 512", 3, 256, 512, 512, False, False),
    ("VAE 256^2 3x3 512->256", 3, 256, 512, 256, False, False),
    ("VAE 256^2 3x3 256 +res", 3, 256, 256, 256, True, False),
    ("VAE 512^2 3x3 256", 3, 512, 256, 256, False, False),
    ("VAE 512^2 3x3 256->128", 3, 512, 256, 128, False, False),
    ("VAE 512^2 3x3 128 +res", 3, 512, 128, 128, True, False),
    ("VAE 512^2 1x1 256->128 +res", 1, 512, 256, 128, True, False),
    ("VAE 256^2 1x1 512->256 +res", 1, 256, 512, 256, True, False),
]
if a.vae:
    SHAPES = VAE_SHAPES
TILES = [int(t) for t in a.tiles.split(",")]
SPLITS = [int(s) for s in a.splits.split(",")]


def graph_us(fn, iters):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / iters * 1e3)
    del g
    return min(ts)


print(f"N = {N}, graph-replayed x{a.iters}", flush=True)
for name, k, h, cin, cout, res, tmb, *c1 in SHAPES:
    if a.only and a.only not in name:
        continue
    c1 = c1[0] if c1 else 0
    h = h if a.vae else h * a.res // 64
    geglu = "geglu" in name
    x = torch.randn(N, h, h, cin, device=dev, dtype=torch.float16)
    x2 = torch.randn(N, h, h, c1, device=dev, dtype=torch.float16) if c1 else None
    w = torch.randn(cout, cin + c1, k, k, device=dev) / math.sqrt(k * k * (cin + c1))
    b = torch.randn(cout, device=dev)
    r = torch.randn(N, h, h, cout, device=dev, dtype=torch.float16) if res else None
    te = torch.randn(N, cout, device=dev, dtype=torch.float16) if tmb else None
    wp, kp = ops.pack_conv_weight(w)
    out = torch.empty(N, h, h, cout // 2 if geglu else cout, device=dev, dtype=torch.float16)
    fn = lambda: ops.conv(x, wp, kp, cout, ksize=k, bias=b, x2=x2, resid=r, temb=te, out=out,  # noqa: E731
                          act="geglu" if geglu else None)
    with ops.force_plan(0, 0):
        with ops.record_conv_plans() as pl:
            fn()
        base = graph_us(fn, a.iters)
    ref = out.float().clone()
    res_t = []
    for t in TILES:
        for sp in SPLITS:
            with ops.force_plan(t, sp):
                with ops.record_conv_plans() as pl2:
                    fn()
                if not pl2 or pl2[0] != (t, sp):
                    continue
                us = graph_us(fn, a.iters)
                err = ((out.float() - ref).norm() / ref.norm()).item()
            res_t.append((us, t, sp, err))
    res_t.sort()
    best = " ".join(f"({t},{s}) {us:.1f}" for us, t, s, _ in res_t[:6])
    emax = max((e for *_, e in res_t), default=0.0)
    print(f"{name:26s} default {pl[0]} {base:7.1f} us | best: {best} | max relerr {emax:.1e}", flush=True)
