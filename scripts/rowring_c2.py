"""c2 (N = 2) level-0 3x3 convs: the planner's plan on the plain source vs the row-ring tile 42 on the
zero-bordered source with K split over channel blocks (forced), graph-replayed device time per call."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")


def graph_us(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
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
    return min(ts)


for n in (2, 8):
    for cin, cout, res, tmb in ((320, 320, True, False), (640, 320, False, True), (960, 320, False, True)):
        h = 64
        xp = torch.zeros(n, h + 2, h + 2, cin, device=dev, dtype=torch.float16)
        xp[:, 1:-1, 1:-1] = torch.randn(n, h, h, cin, device=dev, dtype=torch.float16)
        x = xp[:, 1:-1, 1:-1].contiguous()
        w = torch.randn(cout, cin, 3, 3, device=dev) / math.sqrt(9 * cin)
        b = torch.randn(cout, device=dev)
        r = torch.randn(n, h, h, cout, device=dev, dtype=torch.float16) if res else None
        te = torch.randn(n, cout, device=dev, dtype=torch.float16) if tmb else None
        wp, kp = ops.pack_conv_weight(w)
        out = torch.empty(n, h, h, cout, device=dev, dtype=torch.float16)
        plain = lambda: ops.conv(x, wp, kp, cout, ksize=3, bias=b, resid=r, temb=te, out=out)  # noqa: E731
        padded = lambda: ops.conv(xp, wp, kp, cout, ksize=3, bias=b, resid=r, temb=te, out=out, padded=True)  # noqa: E731
        with ops.record_conv_plans() as pl:
            plain()
        base = graph_us(plain)
        ref = out.float().clone()
        row = [f"N={n} 3x3 {cin}->{cout}: plain {pl[0]} {base:6.1f} us"]
        for sp in (1, 2, 3, 5, 8, 10, 15):
            with ops.force_plan(42, sp):
                with ops.record_conv_plans() as pl2:
                    padded()
                if not pl2 or pl2[0][0] != 42:
                    continue
                us = graph_us(padded)
                err = ((out.float() - ref).norm() / ref.norm()).item()
            row.append(f"(42,{pl2[0][1]}) {us:6.1f} [{err:.1e}]")
        print(" | ".join(row), flush=True)
