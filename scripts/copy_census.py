"""Which host-side calls put device copies (hipMemcpyAsync / copy kernels) into one denoise step?
Runs GraphDenoiser._body() eagerly under torch.profiler (CFG pair, 64^2) and prints every aten op
that launched a copy, with its Python call site.  python scripts/copy_census.py [--batch 1]"""
import argparse
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd.processor import AudioProcessorManager  # noqa: E402
from clap2diffusion_amd.sampler import GraphDenoiser  # noqa: E402
from clap2diffusion_amd.scheduler import DDIMScheduler  # noqa: E402
from clap2diffusion_amd.unet import UNet2DConditionModel  # noqa: E402
from clap2diffusion_amd.weights import synth_unet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1)
a = ap.parse_args()
dev = torch.device("cuda")
unet = UNet2DConditionModel().to(dev)
unet.load_diffusers_state_dict(synth_unet(0, device=dev))
mgr = AudioProcessorManager(unet)
mgr.setup_processors(verbose=False)
for p in mgr.level_processors().values():
    p.to(dev)
N = 2 * a.batch
ehs = torch.randn(N, 77, 768, device=dev, dtype=torch.float16)
audio = {lv: torch.randn(N, 10, 768, device=dev, dtype=torch.float16) for lv in ("early", "mid", "late")}
sched = DDIMScheduler()
sched.set_timesteps(50)
den = GraphDenoiser(unet, sched, a.batch, 64, 64, 7.5, ehs, {"audio": mgr.get_audio_kwargs(audio)}, use_graph=False)
with torch.no_grad():
    den.prepare_context()
    den.x.normal_()
    den._body()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        den._body()
        torch.cuda.synchronize()
sites = collections.Counter()
kinds = collections.Counter()
for ev in prof.events():
    if ev.device_type == torch.autograd.DeviceType.CPU and ev.name in ("aten::copy_", "aten::clone", "aten::contiguous",
                                                                         "aten::cat", "aten::to", "aten::_to_copy"):
        st = [f for f in (ev.stack or []) if "clap2diffusion_amd" in f or "scripts" in f]
        sites[(ev.name, st[0] if st else "?")] += 1
for ev in prof.events():
    if ev.device_type == torch.autograd.DeviceType.CUDA:
        kinds[ev.name[:60]] += 1
print("copy-like aten ops per step (name, innermost package frame):")
for (n, s), c in sites.most_common(40):
    print(f"  {c:4d}  {n:18s} {s}")
print("device activities mentioning copy / memcpy / fill:")
for k, c in kinds.most_common():
    if any(t in k.lower() for t in ("copy", "memcpy", "fill", "memset")):
        print(f"  {c:4d}  {k}")
