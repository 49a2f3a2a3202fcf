"""Per-shape GroupNorm(+SiLU) cost as the UNet sees it: 20 c2d_groupnorm calls captured
in one graph and replayed (no Python launch overhead).  A variant build (-DC2D_TUNE_GN_FUSED_HW=..., loaded
through C2D_LIB) selects the path."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")
N = int(os.environ.get("GN_N", "16"))
SHAPES = [(64, 320, 0), (64, 320, 320), (64, 640, 320), (32, 640, 0), (32, 640, 320), (32, 640, 640), (32, 1280, 640),
          (16, 1280, 0), (16, 1280, 1280),
          (8, 1280, 0), (8, 1280, 1280)]
if os.environ.get("GN_SHAPES") == "vae":   # the VAE decoder's GroupNorms (GN_N=8: c3's batch)
    SHAPES = [(64, 512, 0), (128, 512, 0), (256, 512, 0), (256, 256, 0), (512, 256, 0), (512, 128, 0)]
REPS = 20
for h, c0, c1 in SHAPES:
    x = torch.randn(N, h, h, c0, device=dev, dtype=torch.float16) * 2 + 0.5
    x2 = torch.randn(N, h, h, c1, device=dev, dtype=torch.float16) if c1 else None
    c = c0 + c1
    g = torch.rand(c, device=dev) + 0.5
    b = torch.randn(c, device=dev) * 0.1
    out = torch.empty(N, h, h, c, device=dev, dtype=torch.float16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            ops.group_norm(x, 32, 1e-5, g, b, True, x2=x2, out=out)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(REPS):
            ops.group_norm(x, 32, 1e-5, g, b, True, x2=x2, out=out)
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        graph.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (5 * REPS)
    mb = N * h * h * c * 2 / 1e6
    print(f"GN {h:3d}^2 c={c0}+{c1} ({mb:6.1f} MB): {us:7.1f} us per call", flush=True)
