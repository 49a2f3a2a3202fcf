import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd.pipeline import AudioToImageInference, synthetic_thunder  # noqa: E402
from clap2diffusion_amd.text_encoder import tokenize  # noqa: E402

dev = torch.device("cuda")
use_graph = sys.argv[1] == "graph"
pipe = AudioToImageInference(device=dev, height=128, width=128, verbose=False, use_graph=use_graph)
b = 2
mel = pipe.mel_features([synthetic_thunder(5), synthetic_thunder(6)])
ids = (tokenize([""] * b, dev), tokenize(["a beach"] * b, dev))
lat = pipe.initial_latents([3, 4])


def scan():
    bad = []
    for mname, mod in (("unet", pipe.unet), ("clap", pipe.clap), ("vae", pipe.vae)):
        for n, t in mod.named_buffers():
            if t is not None and t.is_floating_point() and not torch.isfinite(t).all():
                bad.append(f"{mname}.{n}")
    for lv, p in pipe.manager.level_processors().items():
        for k, v in (p._packed or {}).items():
            if torch.is_tensor(v) and not torch.isfinite(v).all():
                bad.append(f"proc.{lv}.{k}")
    return bad


for it in range(4):
    img = pipe.generate_batch(mel, None, 10, 7.5, ids=ids, latents=lat)
    torch.cuda.synchronize()
    den = pipe._denoisers[(b, 10, 7.5)]
    print(it, "x finite", torch.isfinite(den.x).all().item(), "ehs finite", torch.isfinite(den.ehs).all().item(),
          {k: torch.isfinite(v).all().item() for k, v in den.kw["audio"].items()}, "bad buffers", scan()[:8],
          "step", den.step_idx.item(), flush=True)
