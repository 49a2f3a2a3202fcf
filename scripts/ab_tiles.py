"""Same-process A/B of implicit-GEMM plans on chosen shapes: every (shape, plan) pair timed
with HIP events in interleaved rounds (cdna_hip_programming.md §5.4 rule 24), median and min
reported.  Plans are forced through c2d_set_plan_override (ops.force_plan); plan 0 = planner.

python scripts/ab_tiles.py --shapes geglu0,geglu1,geglu2 --plans 0,41:1,25:1 [--rounds 5]
"""
import argparse
import math
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

# name: (ksize, h, cin, cout, act, n, resid)
SHAPES = {
    "geglu0": (1, 64, 320, 2560, "geglu", 16, False),
    "geglu1": (1, 32, 640, 5120, "geglu", 16, False),
    "geglu2": (1, 16, 1280, 10240, "geglu", 16, False),
    "qkv0": (1, 64, 320, 960, None, 16, False),
    "qkv1": (1, 32, 640, 1920, None, 16, False),
    "qkv2": (1, 16, 1280, 3840, None, 16, False),
    "toq0": (1, 64, 320, 320, None, 16, False),
    "toq1": (1, 32, 640, 640, None, 16, False),
    "toq2": (1, 16, 1280, 1280, None, 16, False),
    "proj0": (1, 64, 320, 320, None, 16, True),
    "proj1": (1, 32, 640, 640, None, 16, True),
    "proj2": (1, 16, 1280, 1280, None, 16, True),
    "ff2_0": (1, 64, 1280, 320, None, 16, True),
    "ff2_1": (1, 32, 2560, 640, None, 16, True),
    "ff2_2": (1, 16, 5120, 1280, None, 16, True),
    "conv0": (3, 64, 320, 320, None, 16, True),
    "conv1": (3, 32, 640, 640, None, 16, True),
    "conv2": (3, 16, 1280, 1280, None, 16, True),
    "conv3": (3, 8, 1280, 1280, None, 16, True),
    "upconv3": (3, 8, 2560, 1280, None, 16, False),
    "upconv0": (3, 64, 960, 320, None, 16, False),
    "geglu0_c2": (1, 64, 320, 2560, "geglu", 2, False),
    "conv0_c2": (3, 64, 320, 320, None, 2, True),
    "geglu0_c5": (1, 96, 320, 2560, "geglu", 8, False),
    # zero-bordered sources (c2d_groupnorm_pad -> conv(padded=True)): the row-ring tile 42 at 64^2
    "conv0p": (3, 64, 320, 320, None, 16, True, True),
    "convt0p": (3, 64, 320, 320, None, 16, False, True),
    "upconv0p": (3, 64, 960, 320, None, 16, False, True),
    "conv0_c2p": (3, 64, 320, 320, None, 2, True, True),
}


def make(k, h, cin, cout, act, n, resid, dev, pad=False):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(n, h, h, cin, generator=g).to(dev, torch.float16)
    if pad:
        x = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1)).contiguous()
    w = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(k * k * cin)
    wp, kp = ops.pack_conv_weight(w)
    wp = wp.to(dev)
    b = torch.randn(cout, generator=g).to(dev) * 0.1
    r = torch.randn(n, h, h, cout, generator=g).to(dev, torch.float16) if resid else None
    out = torch.empty(n, h, h, cout // 2 if act == "geglu" else cout, device=dev, dtype=torch.float16)
    return dict(x=x, wp=wp, kp=kp, cout=cout, k=k, b=b, r=r, out=out, act=act, pad=pad,
                flop=2.0 * n * h * h * cout * k * k * cin)


def call(c):
    ops.conv(c["x"], c["wp"], c["kp"], c["cout"], ksize=c["k"], bias=c["b"], act=c["act"], resid=c["r"], out=c["out"],
             padded=c["pad"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="geglu0,geglu1,geglu2")
    ap.add_argument("--plans", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda")
    plans = [tuple(int(v) for v in p.split(":")) if ":" in p else (int(p), 0) for p in a.plans.split(",")]
    cases = {s: make(*SHAPES[s][:7], dev, *SHAPES[s][7:]) for s in a.shapes.split(",")}
    times = {(s, p): [] for s in cases for p in plans}
    used = {}
    outs = {}
    for s, c in cases.items():
        for p in plans:
            with ops.force_plan(*p), ops.record_conv_plans() as rec:
                call(c)
            used[(s, p)] = rec[0] if rec else None
            torch.cuda.synchronize()
            outs[(s, p)] = c["out"].float().clone()
    for _ in range(a.rounds):
        for s, c in cases.items():
            for p in plans:
                with ops.force_plan(*p):
                    call(c)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        call(c)
                    e1.record()
                    e1.synchronize()
                times[(s, p)].append(e0.elapsed_time(e1) / a.iters * 1e3)
    for s, c in cases.items():
        base = outs[(s, plans[0])]
        for p in plans:
            t = times[(s, p)]
            med = statistics.median(t)
            d = (outs[(s, p)] - base).abs().max().item() / max(base.abs().max().item(), 1e-12)
            print(f"{s:10s} plan {p[0]:2d}:{p[1]} ran {used[(s, p)]}  median {med:8.1f} us  min {min(t):8.1f} us  "
                  f"{c['flop'] / med / 1e6:7.1f} TF/s  ({c['flop'] / med / 1e6 / 2500:.3f} of peak)  "
                  f"max diff vs first plan {d:.1e}", flush=True)


if __name__ == "__main__":
    main()
