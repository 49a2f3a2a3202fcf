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

def sums():
    d = {}
    for n, t in pipe.unet.named_buffers():
        if t is not None:
            d["unet." + n] = t.double().abs().sum().item()
    for lv, p in pipe.manager.level_processors().items():
        for k, v in (p._packed or {}).items():
            if torch.is_tensor(v):
                d[f"proc.{lv}.{k}"] = v.double().abs().sum().item()
        for k, v in p.state_dict().items():
            d[f"procsd.{lv}.{k}"] = v.double().abs().sum().item()
    d["ehs"] = den.ehs.double().abs().sum().item()
    for k, v in den.kw["audio"].items():
        d["audio." + k] = v.double().abs().sum().item()
    d["t"] = den.t_table.double().sum().item(); d["coef"] = den.coef.double().sum().item()
    return d

x = den.run(lat); torch.cuda.synchronize()
print("run1", torch.isfinite(x).all().item(), flush=True)
s0 = sums()
q = torch.randn(2, 1, 256, 512, device=dev, dtype=torch.float16)
o = torch.nn.functional.scaled_dot_product_attention(q, q, q); torch.cuda.synchronize()
s1 = sums()
diff = [k for k in s0 if s0[k] != s1[k]]
print("changed after sdpa:", diff[:20], len(diff), flush=True)
x = den.run(lat); torch.cuda.synchronize()
print("run2", torch.isfinite(x).all().item(), flush=True)
s2 = sums()
diff = [k for k in s1 if s1[k] != s2[k]]
print("changed by run2:", diff[:20], len(diff), flush=True)
