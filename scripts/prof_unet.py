"""Scratch profiler: 50-step CFG+DDIM denoise of a batch on the HIP UNet.
python scripts/prof_unet.py --batch 8 --steps 50 [--res 64] [--no-graph]"""
import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd.processor import AudioProcessorManager  # noqa: E402
from clap2diffusion_amd.sampler import GraphDenoiser  # noqa: E402
from clap2diffusion_amd.scheduler import DDIMScheduler  # noqa: E402
from clap2diffusion_amd.unet import UNet2DConditionModel  # noqa: E402
from clap2diffusion_amd.weights import synth_unet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--steps", type=int, default=50)
ap.add_argument("--res", type=int, default=64)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--no-graph", action="store_true")
a = ap.parse_args()
dev = torch.device("cuda")
t0 = time.time()
unet = UNet2DConditionModel().to(dev)
unet.load_diffusers_state_dict(synth_unet(0, device=dev))
mgr = AudioProcessorManager(unet)
mgr.setup_processors(verbose=False)
for p in mgr.level_processors().values():
    p.to(dev)
print(f"setup {time.time() - t0:.1f}s", flush=True)
B = a.batch
ehs = torch.randn(2 * B, 77, 768, device=dev, dtype=torch.float16)
audio = {lv: torch.randn(2 * B, 10, 768, device=dev, dtype=torch.float16) for lv in ("early", "mid", "late")}
sch = DDIMScheduler()
sch.set_timesteps(a.steps)
den = GraphDenoiser(unet, sch, B, a.res, a.res, 7.5, ehs, mgr.get_audio_kwargs(audio), use_graph=not a.no_graph)
lat = torch.randn(B, 4, a.res, a.res, device=dev)
t0 = time.time()
den.run(lat)
torch.cuda.synchronize()
print(f"first run (incl capture) {time.time() - t0:.2f}s", flush=True)
for r in range(a.reps):
    t0 = time.time()
    out = den.run(lat)
    torch.cuda.synchronize()
    dt = time.time() - t0
    print(f"run {r}: {dt:.3f}s  {B / dt:.3f} img/s  {dt / a.steps * 1e3:.2f} ms/step  "
          f"finite={torch.isfinite(out).all().item()} std={out.std().item():.3f}", flush=True)
    if not torch.isfinite(out).all():
        bad = [n for n, b in unet.named_buffers() if b is not None and b.is_floating_point() and not torch.isfinite(b).all()]
        print("non-finite unet buffers:", bad[:10], len(bad))
        for lv, p in mgr.level_processors().items():
            pk = p._packed
            print(lv, {k: torch.isfinite(v).all().item() for k, v in pk.items() if torch.is_tensor(v)})
        print("ehs", torch.isfinite(ehs).all().item(), {k: torch.isfinite(v).all().item() for k, v in audio.items()})
        print("tables", torch.isfinite(den.t_table).all().item(), torch.isfinite(den.coef).all().item(), den.step_idx.item())
        break
