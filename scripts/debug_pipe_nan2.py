import sys
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd.pipeline import AudioToImageInference, synthetic_thunder  # noqa: E402
from clap2diffusion_amd.text_encoder import tokenize  # noqa: E402

dev = torch.device("cuda")
pipe = AudioToImageInference(device=dev, height=128, width=128, verbose=False, use_graph=True)
b = 2
mel = pipe.mel_features([synthetic_thunder(5), synthetic_thunder(6)])
ids = (tokenize([""] * b, dev), tokenize(["a beach"] * b, dev))
lat = pipe.initial_latents([3, 4])
ehs, kw, _ = pipe.condition(mel, ids[0], ids[1])
den = pipe.denoiser(b, 10, 7.5, ehs, kw)
def chk(tag):
    x = den.run(lat); torch.cuda.synchronize()
    print(tag, torch.isfinite(x).all().item(), x.abs().max().item(), flush=True)
chk("run1")
chk("run2")
img = pipe.vae(den.x.clone()); torch.cuda.synchronize()
chk("after vae")
e2, k2, _ = pipe.condition(mel, ids[0], ids[1]); torch.cuda.synchronize()
chk("after condition (no copy)")
den.ehs.copy_(e2)
for k, v in k2["audio"].items():
    den.kw["audio"][k].copy_(v)
chk("after copy of conditioning")
print("ehs diff", (e2.float() - ehs.float()).abs().max().item(), {k: (k2['audio'][k].float()-kw['audio'][k].float()).abs().max().item() for k in k2['audio']})
clap = pipe.clap(mel); torch.cuda.synchronize()
chk("after htsat")
