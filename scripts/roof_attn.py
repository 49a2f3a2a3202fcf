"""Run only the level-0 self-attention (d = 40, 16 CFG images x 8 heads, 4096 queries x 4096
keys: c2d_attention_fwd) so rocprofv3 --pmc passes see exactly that launch.
python scripts/roof_attn.py [iters]"""
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from clap2diffusion_amd import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
# [iters] [L] [images]: the c5 shape (768^2, 96^2 latent, B = 4 -> 8 CFG images) is "5 9216 8"
l = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
b = int(sys.argv[3]) if len(sys.argv) > 3 else 16
h, d = 8, 40
dev = torch.device("cuda:0")
qkv = torch.randn(b * l, 3 * h * d, device=dev, dtype=torch.float16)
c = h * d
out = torch.empty(b * l, c, device=dev, dtype=torch.float16)
for _ in range(2):
    ops.attention(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], b, h, l, l, d, out=out)
s = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(iters):
    ops.attention(qkv[:, :c], qkv[:, c:2 * c], qkv[:, 2 * c:], b, h, l, l, d, out=out)
e1.record(s)
e1.synchronize()
us = e0.elapsed_time(e1) / iters * 1e3
fl = 4.0 * b * h * l * l * d
print(f"attn d={d} L={l}: {us:.1f} us, {fl / us / 1e6:.1f} TF/s", flush=True)
