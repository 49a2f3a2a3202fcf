"""c5 (N = 8, 96^2) level-0 convs whose one-slice grid is one round + a tail: graph-replayed device time
per call and output equality vs the torch fp32 reference; run against the default library and a variant build
(build.py --variant notail --define C2D_TUNE_TAIL_SPLIT=0, loaded through C2D_LIB); TAIL names the arm in the output."""
import math
import os
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

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


torch.manual_seed(0)
for cin, c1, cout, up, res, tmb in ((320, 0, 320, False, True, False), (320, 320, 320, False, False, True),
                                    (640, 320, 320, False, False, True), (640, 0, 640, True, False, False)):
    n, h = 8, 96
    ih = h // 2 if up else h
    x = torch.randn(n, ih, ih, cin, device=dev, dtype=torch.float16)
    x2 = torch.randn(n, ih, ih, c1, device=dev, dtype=torch.float16) if c1 else None
    w = torch.randn(cout, cin + c1, 3, 3, device=dev) / math.sqrt(9 * (cin + c1))
    b = torch.randn(cout, device=dev)
    r = torch.randn(n, h, h, cout, device=dev, dtype=torch.float16) if res else None
    te = torch.randn(n, cout, device=dev, dtype=torch.float16) if tmb else None
    wp, kp = ops.pack_conv_weight(w)
    out = torch.empty(n, h, h, cout, device=dev, dtype=torch.float16)
    fn = lambda: ops.conv(x, wp, kp, cout, ksize=3, bias=b, x2=x2, resid=r, temb=te, out=out, up=up)  # noqa: E731
    us = graph_us(fn)
    xi = torch.cat([x, x2], -1) if c1 else x
    xi = xi.permute(0, 3, 1, 2).float()
    if up:
        xi = F.interpolate(xi, scale_factor=2.0, mode="nearest")
    ref = F.conv2d(xi, w, b, padding=1)
    if te is not None:
        ref = ref + te.float()[:, :, None, None]
    if r is not None:
        ref = ref + r.permute(0, 3, 1, 2).float()
    err = ((out.permute(0, 3, 1, 2).float() - ref).norm() / ref.norm()).item()
    print(f"TAIL={os.environ.get('TAIL', '1')} 3x3 {cin}+{c1}->{cout} up={int(up)}: "
          f"{us:7.1f} us  rel-L2 {err:.2e}", flush=True)
