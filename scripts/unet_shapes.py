"""Per-shape breakdown of the implicit-GEMM calls of one UNet call (CFG batch N = 2B, 64^2 latent).

Records every ops.conv call of one eager UNet forward, then re-runs each unique call
(same tensors, same epilogue) `iters` times between HIP events and prints: count per
UNet call, planned tile / split, us per call, TF/s, and the share of the total.
python scripts/unet_shapes.py [--batch 8] [--res 64] [--iters 10]   (env as usual: C2D_GEMM_TILE ...)"""
import argparse
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

ops.plan_override_from_env()   # C2D_GEMM_TILE / C2D_GEMM_SPLIT (tuning runs only)
from clap2diffusion_amd.processor import AudioProcessorManager  # noqa: E402
from clap2diffusion_amd.unet import UNet2DConditionModel  # noqa: E402
from clap2diffusion_amd.weights import synth_unet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--res", type=int, default=64)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda")
unet = UNet2DConditionModel().to(dev)
unet.load_diffusers_state_dict(synth_unet(0, device=dev))
mgr = AudioProcessorManager(unet)
mgr.setup_processors(verbose=False)
for p in mgr.level_processors().values():
    p.to(dev)
N = 2 * a.batch
x = torch.randn(N, 4, a.res, a.res, device=dev)
ehs = torch.randn(N, 77, 768, device=dev, dtype=torch.float16)
audio = {lv: torch.randn(N, 10, 768, device=dev, dtype=torch.float16) for lv in ("early", "mid", "late")}

calls = []
_conv = ops.conv


def rec(*args, **kw):
    out = _conv(*args, **kw)
    kw = dict(kw)
    kw["out"] = out[0] if isinstance(out, tuple) else out   # (out, GnMoments) when gn_moments > 0
    calls.append((args, kw))
    return out


ops.conv = rec
import clap2diffusion_amd.unet as _u  # noqa: E402
for mod in list(sys.modules.values()):
    if mod is not None and getattr(mod, "__name__", "").startswith("clap2diffusion_amd") and getattr(mod, "conv", None) is _conv:
        mod.conv = rec
with torch.no_grad():
    unet(x, 981, ehs, cross_attention_kwargs={"audio": mgr.get_audio_kwargs(audio)})
torch.cuda.synchronize()
ops.conv = _conv
print(f"{len(calls)} conv / GEMM calls per UNet call (N = {N}, {a.res}^2)", flush=True)


def key(args, kw):
    x, w, kpad, cout = args[:4]
    x2 = kw.get("x2")
    cin = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
    m = x.numel() // x.shape[-1]
    if kw.get("padded"):   # zero-bordered source [n][h + 2][w + 2][c]: output rows n * h * w
        m = x.shape[0] * (x.shape[1] - 2) * (x.shape[2] - 2)
    return (kw["ksize"], m, cin, cout, kw.get("stride", 1), bool(kw.get("up")), kw.get("act"),
            kw.get("resid") is not None, kw.get("temb") is not None, bool(kw.get("padded")))


groups = collections.OrderedDict()
for args, kw in calls:
    groups.setdefault(key(args, kw), []).append((args, kw))

rows = []
for k, lst in groups.items():
    args, kw = lst[0]
    with ops.record_conv_plans() as plans:
        _conv(*args, **kw)
    torch.cuda.synchronize()
    for _ in range(2):
        _conv(*args, **kw)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        _conv(*args, **kw)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    ks, m, cin, cout, st, up, act, res, temb, pad = k
    oh_m = m if ks == 1 else m // (st * st) * (4 if up else 1)
    fl = 2.0 * oh_m * cout * ks * ks * cin
    rows.append((k, len(lst), plans[0] if plans else None, us, fl))

tot = sum(c * us for _, c, _, us, _ in rows)
print(f"total {tot / 1e3:.2f} ms per UNet call in conv / GEMM")
for k, c, pl, us, fl in sorted(rows, key=lambda r: -r[1] * r[3]):
    ks, m, cin, cout, st, up, act, res, temb, pad = k
    tag = f"{'3x3' if ks == 3 else '1x1'} M={m:6d} {cin:4d}->{cout:5d}" + (f" s{st}" if st > 1 else "") + \
          (" up" if up else "") + (" pad" if pad else "") + (f" {act}" if act else "") + (" +res" if res else "") + (" +temb" if temb else "")
    print(f"{tag:48s} x{c:2d} plan={pl} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s  {100 * c * us / tot:5.1f}%", flush=True)
