"""Row-ring 3x3 tiles (42 / 43 / 44, igemm_pp16r.h) against the planner's other plans on the
UNet's stride-1 3x3 shapes over the zero-bordered source, graph-replayed device time per call and
rel-L2 against torch fp32.  python scripts/rowring_ab.py [--batch 8] [--iters 20]
Each line: shape, plan (tile, split) as run, us per call, rel-L2."""
import argparse
import math
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

SHAPES_C2 = [  # N = 2 (c2): the planner's table plans against the row-ring tiles with split K
    ("c2 L0 3x3 320 +res", 64, 320, 320, "resid", [(7, 4), (42, 5), (42, 3)]),
    ("c2 L0 3x3 960->320 +temb", 64, 960, 320, "temb", [(40, 8), (42, 8), (42, 15)]),
    ("c2 L1 3x3 640 +res", 32, 640, 640, "resid", [(7, 8), (43, 4), (43, 8), (43, 10)]),
    ("c2 L1 3x3 1920->640 +temb", 32, 1920, 640, "temb", [(40, 16), (43, 8), (43, 15)]),
    ("c2 L2 3x3 1280 +res", 16, 1280, 1280, "resid", [(7, 12), (44, 8), (44, 10), (44, 20)]),
]
SHAPES = [  # name, h, cin, cout, form, plans to force (tile, split)
    ("L0 3x3 320 +res", 64, 320, 320, "resid", [(40, 1), (42, 1)]),
    ("L1 3x3 640 +res", 32, 640, 640, "resid", [(40, 2), (43, 1), (43, 2), (7, 1)]),
    ("L1 3x3 640 +temb", 32, 640, 640, "temb", [(40, 2), (43, 1)]),
    ("L1 3x3 1920->640 +temb", 32, 1920, 640, "temb", [(40, 2), (43, 1), (43, 2)]),
    ("L1 3x3 960->640 +temb", 32, 960, 640, "temb", [(40, 2), (43, 1)]),
    ("L1 3x3 320->640 +temb", 32, 320, 640, "temb", [(7, 1), (43, 1)]),
    ("L2 3x3 1280 +res", 16, 1280, 1280, "resid", [(40, 4), (44, 2), (44, 3), (44, 4), (44, 1)]),
    ("L2 3x3 2560->1280 +temb", 16, 2560, 1280, "temb", [(40, 4), (44, 2), (44, 4)]),
    ("L2 3x3 640->1280 +temb", 16, 640, 1280, "temb", [(40, 4), (44, 2), (44, 4)]),
]


def gen(*shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):   # clocks up, caches warm
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated name substrings")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = 2 * a.batch
    for name, h, cin, cout, form, plans in (SHAPES_C2 if a.batch == 1 else SHAPES):
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        x = gen(N, cin, h, h, seed=1)
        w = gen(cout, cin, 3, 3, seed=2, scale=1 / math.sqrt(9 * cin))
        b = gen(cout, seed=3) * 0.1
        ref = F.conv2d(x, w, b, padding=1)
        temb = resid = None
        if form == "temb":
            temb = gen(N, cout, seed=4)
            ref = ref + temb[:, :, None, None]
        else:
            resid = gen(N, cout, h, h, seed=5)
            ref = ref + resid
        xp = torch.zeros(N, h + 2, h + 2, cin)
        xp[:, 1:-1, 1:-1] = x.permute(0, 2, 3, 1)
        xp = xp.half().to(dev)
        wp, kp = ops.pack_conv_weight(w)
        wp, bd = wp.to(dev), b.float().to(dev)
        td = None if temb is None else temb.half().to(dev)
        rd = None if resid is None else resid.permute(0, 2, 3, 1).contiguous().half().to(dev)
        out = torch.empty(N, h, h, cout, dtype=torch.float16, device=dev)
        refn = ref.permute(0, 2, 3, 1).to(dev)
        for pl in [None] + plans:
            def run():
                ops.conv(xp, wp, kp, cout, ksize=3, bias=bd, padded=True, temb=td, resid=rd, out=out)
            try:
                if pl is None:
                    with ops.record_conv_plans() as rec:
                        run()
                    us = timed(run, a.iters)
                else:
                    with ops.force_plan(*pl):
                        with ops.record_conv_plans() as rec:
                            run()
                        us = timed(run, a.iters)
            except Exception as e:  # noqa: BLE001
                print(f"{name:28s} {str(pl):10s} failed: {e}", flush=True)
                continue
            err = ((out.float() - refn).norm() / refn.norm()).item()
            tag = "planner" if pl is None else "forced"
            print(f"{name:28s} {tag:8s} {str(rec[0]):10s} {us:8.1f} us  rel-L2 {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
