import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
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
B = 8
torch.manual_seed(0)
ehs = torch.randn(2 * B, 77, 768, device=dev, dtype=torch.float16)
audio = {lv: torch.randn(2 * B, 10, 768, device=dev, dtype=torch.float16) for lv in ("early", "mid", "late")}
sch = DDIMScheduler()
sch.set_timesteps(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
lat = torch.randn(B, 4, 64, 64, device=dev)
den = GraphDenoiser(unet, sch, B, 64, 64, 7.5, ehs, mgr.get_audio_kwargs(audio), use_graph=True)
outs = [den.run(lat).clone() for _ in range(3)]
print("A no-inspect:", [torch.isfinite(o).all().item() for o in outs], flush=True)
for i in range(3):
    o = den.run(lat)
    print("B inspect:", i, torch.isfinite(o).all().item(), o.std().item(), flush=True)
junk = torch.full((1 << 28,), float("nan"), device=dev)
del junk
for i in range(2):
    o = den.run(lat)
    print("C after nan-fill:", i, torch.isfinite(o).all().item(), flush=True)
    junk = torch.full((1 << 28,), float("nan"), device=dev)
    del junk
