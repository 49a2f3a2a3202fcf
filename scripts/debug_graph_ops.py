"""Which HIP op misbehaves when replayed from a hipGraph after unrelated eager work?"""
import math
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)


def disturb():
    q = torch.randn(2, 1, 4096, 512, device=dev, dtype=torch.float16)
    F.scaled_dot_product_attention(q, q, q)
    torch.isfinite(q).all().item()
    q.std().item()
    torch.cuda.synchronize()


def test(name, fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ref = fn().clone()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    res = []
    for i in range(4):
        g.replay()
        torch.cuda.synchronize()
        res.append((out.float() - ref.float()).abs().max().item())
        disturb()
    print(f"{name:28s} replay-vs-eager max|diff| per replay: {res}", flush=True)


x = torch.randn(4, 32, 32, 320, device=dev, dtype=torch.float16)
g_, b_ = torch.ones(320, device=dev) * 1.1, torch.zeros(320, device=dev) + 0.1
w, kp = ops.pack_conv_weight(torch.randn(320, 320, 3, 3, device=dev) / math.sqrt(2880))
test("conv3x3", lambda: ops.conv(x, w, kp, 320, ksize=3))
test("gn_stats(scale)", lambda: ops.group_norm_stats(x, 32, 1e-5, g_, b_)[0])
test("gn+conv", lambda: ops.conv(x, w, kp, 320, ksize=3, gn=ops.group_norm_stats(x, 32, 1e-5, g_, b_), gn_silu=True))
x2 = x.view(-1, 320)
test("layer_norm", lambda: ops.layer_norm(x2, g_, b_, 1e-5))
st = lambda: ops.layer_norm_stats(x2, 1e-5)  # noqa: E731
wl, kl = ops.pack_linear_weight(torch.randn(960, 320, device=dev) / math.sqrt(320))
test("ln-prologue gemm", lambda: ops.conv(x2, wl, kl, 960, ksize=1, ln=(st(), g_, b_)))
qkv = ops.conv(x2, wl, kl, 960, ksize=1)
test("attention d40", lambda: ops.attention(qkv[:, :320], qkv[:, 320:640], qkv[:, 640:], 4, 8, 1024, 1024, 40))
kv = torch.randn(4 * 77, 640, device=dev, dtype=torch.float16)
test("cross attention", lambda: ops.attention(qkv[:, :320], kv[:, :320], kv[:, 320:], 4, 8, 1024, 77, 40))
tt = torch.tensor([981.0, 961.0], device=dev)
si = torch.zeros(1, dtype=torch.int32, device=dev)
test("timestep emb", lambda: ops.timestep_embedding(tt, si, 4, 320))
test("row_mean", lambda: ops.row_mean(x2, 4, 1024))
