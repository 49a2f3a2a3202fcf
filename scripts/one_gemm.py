"""Run one GEMM/conv shape repeatedly (for rocprofv3 counter collection)."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ops.plan_override_from_env()   # C2D_GEMM_TILE / C2D_GEMM_SPLIT (tuning runs only)

k, h, cin, cout = (int(a) for a in sys.argv[1:5])
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
N = 16
dev = torch.device("cuda")
x = torch.randn(N, h, h, cin, device=dev, dtype=torch.float16)
w = torch.randn(cout, cin, k, k, device=dev) / math.sqrt(k * k * cin)
wp, kp = ops.pack_conv_weight(w)
out = torch.empty(N, h, h, cout, device=dev, dtype=torch.float16)
for _ in range(iters):
    ops.conv(x, wp, kp, cout, ksize=k, out=out)
torch.cuda.synchronize()
print("done")
