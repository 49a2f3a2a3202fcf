"""Per-shape timing of c2d_attention_fwd on the UNet's attention shapes (CFG batch 16, 8 heads)."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")
SHAPES = [  # name, batch, heads, lq, lk, d
    ("L0 self 4096x4096 d40", 16, 8, 4096, 4096, 40),
    ("c2 L0 self 4096x4096 d40", 2, 8, 4096, 4096, 40),     # 512^2, B = 1 with CFG
    ("c2 prefix self 4096x4096 d40", 1, 8, 4096, 4096, 40),   # the CFG-shared first self-attention
    ("c5 L0 self 9216x9216 d40", 8, 8, 9216, 9216, 40),   # 768^2, B = 4 with CFG
    ("L0 cross 4096x77 d40", 16, 8, 4096, 77, 40),
    ("L1 self 1024x1024 d80", 16, 8, 1024, 1024, 80),
    ("L2 self 256x256 d160", 16, 8, 256, 256, 160),
    ("L1 cross 1024x77 d80", 16, 8, 1024, 77, 80),
    ("L2 cross 256x77 d160", 16, 8, 256, 77, 160),
]


def run(name, b, h, lq, lk, d, iters=10):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(b * lq, h * d, device=dev, generator=g).half()
    k = torch.randn(b * lk, h * d, device=dev, generator=g).half()
    v = torch.randn(b * lk, h * d, device=dev, generator=g).half()
    o = torch.empty_like(q)
    call = lambda: ops.attention(q, k, v, b, h, lq, lk, d, out=o)  # noqa: E731
    for _ in range(2):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    fl = 4.0 * b * h * lq * lk * d
    qh = q.view(b, lq, h, d).transpose(1, 2)[:2].float()
    kh = k.view(b, lk, h, d).transpose(1, 2)[:2].float()
    vh = v.view(b, lk, h, d).transpose(1, 2)[:2].float()
    ref = F.scaled_dot_product_attention(qh, kh, vh).transpose(1, 2).reshape(min(b, 2), lq, h * d)
    err = ((o.view(b, lq, h * d)[:2].float() - ref).norm() / ref.norm()).item()
    print(f"{name:24s} {ms * 1e3:9.1f} us {fl / ms / 1e9:8.1f} TF/s  relerr {err:.1e}", flush=True)


for s in SHAPES:
    run(*s)
