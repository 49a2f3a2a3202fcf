import sys
from pathlib import Path
import torch
import torch.nn.functional as F
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402
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
    return torch.isfinite(x).all().item()
chk("run1")
mode = sys.argv[1]
if mode == "sdpa":
    q = torch.randn(2, 1, 256, 512, device=dev, dtype=torch.float16)
    o = F.scaled_dot_product_attention(q, q, q); torch.cuda.synchronize()
    chk("after sdpa small")
    q = torch.randn(2, 1, 4096, 512, device=dev, dtype=torch.float16)
    o = F.scaled_dot_product_attention(q, q, q); torch.cuda.synchronize()
    chk("after sdpa 4096")
elif mode == "gn":
    x = torch.randn(2, 64, 64, 512, device=dev, dtype=torch.float16)
    g = torch.ones(512, device=dev); bb = torch.zeros(512, device=dev)
    sc = ops.group_norm_stats(x, 32, 1e-6, g, bb); torch.cuda.synchronize()
    chk("after gn stats")
elif mode == "conv":
    x = torch.randn(2, 64, 64, 512, device=dev, dtype=torch.float16)
    w, kp = ops.pack_conv_weight(torch.randn(512, 512, 3, 3, device=dev) * 0.01)
    y = ops.conv(x, w, kp, 512, ksize=3); torch.cuda.synchronize()
    chk("after conv")
elif mode == "unet":
    with torch.no_grad():
        e = pipe.unet(lat, 981, ehs[:2]).sample; torch.cuda.synchronize()
    chk("after eager unet")
elif mode == "vae":
    pipe.vae(den.x.clone()); torch.cuda.synchronize()
    chk("after vae")
