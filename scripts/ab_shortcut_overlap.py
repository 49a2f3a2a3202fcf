"""Same-process A/B of ResnetBlock2D.overlap_shortcut (the 1x1 shortcut on a side stream) on the
bench's c3 workload (B = 8, 512^2, 50 steps, BatchGraph): the graphs are re-captured per
setting, settings alternate, and the images of the two settings must be bit-identical.
python scripts/ab_shortcut_overlap.py [--reps 2]"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import distributed as D  # noqa: E402
from clap2diffusion_amd.pipeline import AudioToImageInference  # noqa: E402
from clap2diffusion_amd.unet import ResnetBlock2D  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda")
pipe = AudioToImageInference(device=dev, height=512, width=512, verbose=False)
inp = D.rank_inputs(range(8), (64, 64), dev)
clips = pipe.feature_extractor.crop(inp.audios)
wave = torch.from_numpy(np.concatenate(clips)).to(dev)
lens = torch.tensor([c.size for c in clips], dtype=torch.int32, device=dev)
offs = torch.tensor(np.cumsum([0] + [c.size for c in clips[:-1]]), dtype=torch.int64, device=dev)


def run(overlap: bool, n: int = 2):
    ResnetBlock2D.overlap_shortcut = overlap
    pipe._batch_graphs.clear()
    img = pipe.generate_batch_graphed(wave, offs, lens, (inp.ids_uncond, inp.ids_cond), inp.latents, 50, 7.5)
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(n):
        img = pipe.generate_batch_graphed(wave, offs, lens, (inp.ids_uncond, inp.ids_cond), inp.latents, 50, 7.5)
    torch.cuda.synchronize()
    return 8 * n / (time.time() - t0), img.clone()


ref = None
for r in range(a.reps):
    for ov in (False, True):
        ips, img = run(ov)
        same = "" if ref is None else f" images == serial: {bool(torch.equal(img, ref))}"
        if not ov and ref is None:
            ref = img
        print(f"rep {r} overlap_shortcut={ov}: {ips:.3f} images/s{same}", flush=True)
