"""Graph-replayed timing of one conv / GEMM shape through ops.conv, with the max error
against a torch fp32 reference (A/B of library variants: C2D_LIB=... TAG=...).
python scripts/time_gemm.py k h cin cout [--n N] [--geglu] [--res] [--iters I]"""
import argparse
import math
import os
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("k", type=int)
ap.add_argument("h", type=int)
ap.add_argument("cin", type=int)
ap.add_argument("cout", type=int)
ap.add_argument("--n", type=int, default=16)
ap.add_argument("--geglu", action="store_true")
ap.add_argument("--res", action="store_true")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
k, h, cin, cout, N = a.k, a.h, a.cin, a.cout, a.n
torch.manual_seed(0)
dev = torch.device("cuda")
x = torch.randn(N, h, h, cin, device=dev, dtype=torch.float16)
w = torch.randn(cout, cin, k, k, device=dev) / math.sqrt(k * k * cin)
b = torch.randn(cout, device=dev) * 0.1
if a.geglu:
    wi, bi = ops.geglu_interleave(w[:, :, 0, 0].float(), b)
    wp, kp = ops.pack_linear_weight(wi)
    bk = bi.float()
else:
    wp, kp = ops.pack_conv_weight(w)
    bk = b
oc = cout // 2 if a.geglu else cout
out = torch.empty(N, h, h, oc, device=dev, dtype=torch.float16)
r = torch.randn(N, h, h, oc, device=dev, dtype=torch.float16) if a.res else None
act = "geglu" if a.geglu else None


def run():
    ops.conv(x, wp, kp, cout, ksize=k, bias=bk, resid=r, act=act, out=out)


run()
torch.cuda.synchronize()
ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), b.float(), padding=k // 2).permute(0, 2, 3, 1)
if a.geglu:
    hh, gg = ref.chunk(2, dim=-1)
    ref = hh * F.gelu(gg)
if r is not None:
    ref = ref + r.float()
err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    run()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(a.iters):
        run()
g.replay()
torch.cuda.synchronize()
ts = []
for _ in range(7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1) * 1000 / a.iters)
ts.sort()
flop = 2.0 * N * h * h * cout * cin * k * k
print(f"{os.environ.get('TAG', '')} k{k} {h}^2 {cin}->{cout}{' geglu' if a.geglu else ''} N={N}: "
      f"median {ts[3]:.1f} us min {ts[0]:.1f} us  {flop / ts[3] / 1e6:.1f} TF/s  max err/max {err:.2e}")
