"""Run one GEMM/conv shape repeatedly (for rocprofv3 counter collection).
python scripts/one_gemm.py k h cin cout [iters] [--res] [--geglu] [--n N] [--pad]"""
import argparse
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ops.plan_override_from_env()   # C2D_GEMM_TILE / C2D_GEMM_SPLIT (tuning runs only)

ap = argparse.ArgumentParser()
ap.add_argument("k", type=int)
ap.add_argument("h", type=int)
ap.add_argument("cin", type=int)
ap.add_argument("cout", type=int)
ap.add_argument("iters", type=int, nargs="?", default=10)
ap.add_argument("--res", action="store_true")
ap.add_argument("--geglu", action="store_true")
ap.add_argument("--n", type=int, default=16)
ap.add_argument("--pad", action="store_true", help="zero-bordered source (conv padded=True, tile 42)")
a = ap.parse_args()
k, h, cin, cout, N = a.k, a.h, a.cin, a.cout, a.n
dev = torch.device("cuda")
x = torch.randn(N, h, h, cin, device=dev, dtype=torch.float16)
if a.pad:
    x = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1)).contiguous()
w = torch.randn(cout, cin, k, k, device=dev) / math.sqrt(k * k * cin)
b = torch.randn(cout, device=dev)
if a.geglu:
    wi, bi = ops.geglu_interleave(w[:, :, 0, 0].float(), b)
    wp, kp = ops.pack_linear_weight(wi)
    b = bi.float()
else:
    wp, kp = ops.pack_conv_weight(w)
oc = cout // 2 if a.geglu else cout
out = torch.empty(N, h, h, oc, device=dev, dtype=torch.float16)
r = torch.randn(N, h, h, oc, device=dev, dtype=torch.float16) if a.res else None
for _ in range(a.iters):
    ops.conv(x, wp, kp, cout, ksize=k, bias=b, resid=r, act="geglu" if a.geglu else None, out=out, padded=a.pad)
torch.cuda.synchronize()
print("done")
