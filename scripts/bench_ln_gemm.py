"""LayerNorm -> projection GEMM at the c2 / c3 shapes, graph-replayed: (a) c2d_layernorm + the planner's
GEMM (what unet.py runs), (b) c2d_layernorm_stats + the register-staged GEMM with the C2D_PRO_LN
prologue (normalisation applied while staging A), max |diff| between them.
python scripts/bench_ln_gemm.py [--n 2]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda")
N = a.n
SHAPES = [  # (name, rows per image, C, cout, act)
    ("L0 qkv", 4096, 320, 960, None), ("L0 to_q", 4096, 320, 320, None), ("L0 geglu", 4096, 320, 2560, "geglu"),
    ("L1 qkv", 1024, 640, 1920, None), ("L1 to_q", 1024, 640, 640, None), ("L1 geglu", 1024, 640, 5120, "geglu"),
    ("L2 qkv", 256, 1280, 3840, None), ("L2 to_q", 256, 1280, 1280, None), ("L2 geglu", 256, 1280, 10240, "geglu"),
    ("mid qkv", 64, 1280, 3840, None), ("mid geglu", 64, 1280, 10240, "geglu"),
]
REPS = 20


def timed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(REPS):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (5 * REPS)


for name, rows, c, cout, act in SHAPES:
    m = N * rows
    x = (torch.randn(m, c, device=dev) * 2 + 0.5).half()
    gam = torch.rand(c, device=dev) + 0.5
    bet = torch.randn(c, device=dev) * 0.1
    w = torch.randn(cout, c, device=dev) / math.sqrt(c)
    b = torch.randn(cout, device=dev) * 0.1 if act == "geglu" else None
    if act == "geglu":
        w, b = ops.geglu_interleave(w, b)
    wp, kp = ops.pack_linear_weight(w)
    oc = cout // 2 if act == "geglu" else cout
    out_a = torch.empty(m, oc, device=dev, dtype=torch.float16)
    out_b = torch.empty_like(out_a)
    y = torch.empty_like(x)

    def fa():
        ops.layer_norm(x, gam, bet, 1e-5, out=y)
        ops.conv(y, wp, kp, cout, ksize=1, bias=b, act=act, out=out_a)

    def fb():
        st = ops.layer_norm_stats(x, 1e-5)
        ops.conv(x, wp, kp, cout, ksize=1, bias=b, act=act, out=out_b, ln=(st, gam, bet))

    with ops.record_conv_plans() as pa:
        fa()
    with ops.record_conv_plans() as pb:
        fb()
    ta, tb = timed(fa), timed(fb)
    torch.cuda.synchronize()
    d = (out_a.float() - out_b.float()).abs().max().item()
    print(f"{name:10s} M={m:6d} {c:5d}->{cout:6d}  LN+GEMM{pa[0]} {ta:7.1f} us   stats+LN-prologue GEMM{pb[0]} "
          f"{tb:7.1f} us   max|diff| {d:.2e}", flush=True)
