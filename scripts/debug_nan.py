import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402
from clap2diffusion_amd.processor import AudioProcessorManager  # noqa: E402
from clap2diffusion_amd.sampler import GraphDenoiser  # noqa: E402
from clap2diffusion_amd.scheduler import DDIMScheduler  # noqa: E402
from clap2diffusion_amd.unet import UNet2DConditionModel  # noqa: E402
from clap2diffusion_amd.weights import synth_unet  # noqa: E402

dev = torch.device("cuda")
unet = UNet2DConditionModel().to(dev)
unet.load_diffusers_state_dict(synth_unet(0, device=dev))
mgr = AudioProcessorManager(unet)
mgr.setup_processors(verbose=False)
for p in mgr.level_processors().values():
    p.to(dev)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
torch.manual_seed(0)
ehs = torch.randn(2 * B, 77, 768, device=dev, dtype=torch.float16)
audio = {lv: torch.randn(2 * B, 10, 768, device=dev, dtype=torch.float16) for lv in ("early", "mid", "late")}
sch = DDIMScheduler()
sch.set_timesteps(50)
lat = torch.randn(B, 4, 64, 64, device=dev)

# hook: max |activation| at every HIP conv output
maxes = []
orig = ops.conv


def conv_hook(*a, **k):
    out = orig(*a, **k)
    maxes.append(out.float().abs().max().item())
    return out


den = GraphDenoiser(unet, sch, B, 64, 64, 7.5, ehs, mgr.get_audio_kwargs(audio), use_graph=False)
den.x.copy_(lat)
den.step_idx.zero_()
ops.conv = conv_hook
import clap2diffusion_amd.layers as L  # noqa: E402
import clap2diffusion_amd.processor as P  # noqa: E402
import clap2diffusion_amd.unet as U  # noqa: E402
L.ops.conv = conv_hook
with torch.no_grad():
    for s in range(50):
        maxes.clear()
        den._body()
        torch.cuda.synchronize()
        x = den.x
        print(f"step {s}: max|x|={x.abs().max().item():.3f} finite={torch.isfinite(x).all().item()} "
              f"max conv out={max(maxes):.1f} nconv={len(maxes)}", flush=True)
        if not torch.isfinite(x).all():
            break
ops.conv = orig
L.ops.conv = orig
eager = den.x.clone()
den2 = GraphDenoiser(unet, sch, B, 64, 64, 7.5, ehs, mgr.get_audio_kwargs(audio), use_graph=True)
r1 = den2.run(lat).clone()
r2 = den2.run(lat).clone()
r3 = den2.run(lat).clone()
print("graph finite", [torch.isfinite(r).all().item() for r in (r1, r2, r3)])
print("eager vs graph", (eager - r1).abs().max().item(), (r1 - r2).abs().max().item(), (r2 - r3).abs().max().item())
