#!/usr/bin/env python3
"""Benchmark: 512x512 images/sec @ 50 DDIM steps, batch 8 per GPU (BASELINE.json metric).

One bench "step" = one full generation of a batch of 8 images on every rank:
CLAP log-mel (HIP) -> HTSAT (HIP) -> audio projectors -> CLIP text tower -> 50 CFG+DDIM denoise steps of
the audio-conditioned SD1.5 UNet (HIP kernels, replayed hipGraph) -> VAE decode
-> RCCL all-gather of the uint8 images to every rank.  Inputs (48 kHz waveforms,
token ids, per-sample seeded latents) are resident in HBM before the timed
region.  Synthetic inputs and seeded random weights of the SD1.5 / CLAP HTSAT
architectures (no network, no checkpoints).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_F16_TFLOPS = 2500.0  # MI355X dense fp16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
UNET_GFLOP_PER_SAMPLE = 803.2  # SURVEY.md Appendix C, 64x64 latent


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def measure_dominant_kernel(dev, iters: int = 20):
    """The dominant kernel is the implicit-GEMM conv (c2d_conv2d_igemm): time its
    most frequent heavy launch, the level-0 ResnetBlock2D conv (320 -> 320, 3x3,
    N = 16 CFG images, 64x64) with HIP events on the stream it is launched on."""
    from clap2diffusion_amd import ops
    n, h, c = 16, 64, 320
    x = torch.randn(n, h, h, c, device=dev, dtype=torch.float16)
    w = torch.randn(c, c, 3, 3, device=dev) / math.sqrt(9 * c)
    wp, kp = ops.pack_conv_weight(w)
    b = torch.zeros(c, device=dev)
    res = torch.randn_like(x)
    out = torch.empty_like(x)
    for _ in range(3):
        ops.conv(x, wp, kp, c, ksize=3, bias=b, resid=res, out=out)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        ops.conv(x, wp, kp, c, ksize=3, bias=b, resid=res, out=out)
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flop = 2.0 * n * h * h * c * (9 * c)
    tflops = flop / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tflops / PEAK_F16_TFLOPS, 4), "traffic": None,
            "kernel": "c2d_conv2d_igemm (igemm_m32_kernel 256x320 tile) level-0 ResnetBlock2D conv 3x3 320->320 + residual, "
                      "N=16 (CFG pair x 8 images) x 64x64",
            "flop_per_launch": flop, "avg_us": round(ms * 1e3, 2)}


def pmc_traffic(timeout_s: int = 120):
    """HBM bytes per launch of the dominant kernel from rocprofv3 PMC counters, one
    counter per pass (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE (KiB, reported
    at half the bytes of wide streaming reads on gfx950, so doubled) + WRITE_SIZE
    (KiB, exact for 16-B/lane stores).  The passes run scripts/roof_kernel.py (the
    same launch as measure_dominant_kernel) in a child process; None if rocprofv3
    is unavailable or a pass fails."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    vals = {}
    with tempfile.TemporaryDirectory() as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(td, ctr)
            cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
                   sys.executable, str(ROOT / "scripts" / "roof_kernel.py"), "4"]
            try:
                subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=timeout_s,
                               check=True)
            except Exception as e:  # noqa: BLE001 - reported, never fatal to the bench
                return None, f"{ctr} pass failed: {type(e).__name__}"
            got = []
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        for r in csv.DictReader(open(os.path.join(root, f))):
                            if "igemm" in r["Kernel_Name"] and r["Counter_Name"] == ctr:
                                got.append(float(r["Counter_Value"]))
            if not got:
                return None, f"{ctr}: no igemm rows"
            got.sort()
            vals[ctr] = got[len(got) // 2]
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, f"rocprofv3 --pmc: FETCH_SIZE {vals['FETCH_SIZE']:.0f} KiB (x2, gfx950) + WRITE_SIZE " \
                    f"{vals['WRITE_SIZE']:.0f} KiB per launch"


def cpu_baseline(calls: int = 2):
    """The fp32 CPU oracle (oracle/unet_ref.py, a port of the diffusers path the
    reference glues together) timed on host cores: `calls` CFG-pair UNet calls at
    512x512 (64x64 latent, N = 2), extrapolated to images/sec at 50 DDIM steps."""
    from clap2diffusion_amd.weights import synth_unet
    from oracle.unet_ref import UNetRef
    cores = min(16, os.cpu_count() or 1)
    torch.set_num_threads(cores)
    ref = UNetRef(synth_unet(0))
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 4, 64, 64, generator=g)
    ehs = torch.randn(2, 77, 768, generator=g)
    with torch.no_grad():
        ref(x, 981, ehs)  # warm-up
        t0 = time.time()
        for i in range(calls):
            ref(x, 981 - 20 * i, ehs)
        dt = (time.time() - t0) / calls
    return {"value": round(1.0 / (dt * 50), 6), "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": f"{calls} UNet calls (CFG pair, fp32, 64x64 latent) on {cores} threads = {dt:.2f} s/call, "
                      f"x50 DDIM steps per image; HTSAT/CLIP/VAE excluded (they add ~3% of the FLOPs)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2, help="timed batch generations")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU")
    ap.add_argument("--ddim-steps", type=int, default=50)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from clap2diffusion_amd.pipeline import AudioToImageInference, synthetic_thunder
    from clap2diffusion_amd.text_encoder import tokenize

    t_setup = time.time()
    pipe = AudioToImageInference(device=dev, height=a.res, width=a.res, verbose=False)
    B = a.batch
    gidx = [rank * B + i for i in range(B)]  # global sample indices of this rank
    audios = [synthetic_thunder(i) for i in gidx]
    # waveforms resident in HBM; the log-mel front end (c2d_clap_log_mel) runs inside the step
    clips = pipe.feature_extractor.crop(audios)
    wave = torch.from_numpy(np.concatenate(clips)).to(dev)
    lens = torch.tensor([c.size for c in clips], dtype=torch.int32, device=dev)
    offs = torch.tensor(np.cumsum([0] + [c.size for c in clips[:-1]]), dtype=torch.int64, device=dev)
    prompts = ["a beach" if i % 2 == 0 else "a city street at night" for i in gidx]
    ids = (tokenize([""] * B, dev), tokenize(prompts, dev))
    latents = pipe.initial_latents([i for i in gidx])
    gathered = [torch.empty(B, a.res, a.res, 3, dtype=torch.uint8, device=dev) for _ in range(world)]
    if rank == 0:
        log(f"[bench] setup {time.time() - t_setup:.1f}s, world={world}, batch/gpu={B}")

    def one_batch():
        mel = pipe.feature_extractor.from_device(wave, offs, lens)
        img = pipe.generate_batch(mel, None, a.ddim_steps, 7.5, ids=ids, latents=latents)
        if world > 1:
            dist.all_gather(gathered, img)
        else:
            gathered[0] = img
        return img

    for i in range(a.warmup):
        one_batch()
        torch.cuda.synchronize()
        if rank == 0:
            log(f"[bench] warmup {i} done")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        img = one_batch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    finite = bool(torch.isfinite(pipe._denoisers[(B, a.ddim_steps, 7.5)].x).all().item())
    ms_per_step = dt / a.steps * 1e3
    total_images = world * B * a.steps
    value = total_images / dt

    if rank == 0:
        roof = measure_dominant_kernel(dev)
        unet_tf = UNET_GFLOP_PER_SAMPLE * (a.res / 512) ** 2 * 2 * a.ddim_steps * world * B * a.steps / dt / 1e3
        roof["pipeline_unet_tflops"] = round(unet_tf, 2)
        n_, h_, c_ = 16, 64, 320
        roof["algorithmic_bytes"] = 2 * (3 * n_ * h_ * h_ * c_ + c_ * 9 * c_)  # x + resid + out + weights
        if not a.no_pmc and world == 1:
            tr, src = pmc_traffic()
            roof["traffic"] = None if tr is None else round(tr)
            roof["traffic_source"] = src
        cpu = None if (a.no_cpu_baseline or world > 1) else cpu_baseline()
        # BASELINE.json configs: c3 is the default line; other shapes are labelled, not the metric
        cfg_name = {(512, 8): "c3", (512, 1): "c2", (768, 4): "c5"}.get((a.res, B), "custom")
        if world > 1 and (a.res, B) == (512, 8):
            cfg_name = "c4" if world == 8 else "c3-sharded"
        line = {
            "metric": "512x512 images/sec @ 50 DDIM steps, batch=8, 1/2/4/8 MI355X",
            "value": round(value, 4), "unit": "images/sec", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp16",
            "data": "synthetic (seeded thunder-like audio, fixed token ids, random-init SD1.5/CLAP weights)",
            "config": {"workload": f"{cfg_name}: batch={B}/GPU, {a.ddim_steps} DDIM steps, {a.res}x{a.res}, CFG 7.5, "
                                   "log-mel+HTSAT+projectors+CLIP+UNet+VAE, all-gather of images",
                       "global_batch": B * world, "ddim_steps": a.ddim_steps, "resolution": a.res,
                       "parallelism": f"dp{world}"},
            "roofline": roof, "cpu_baseline": cpu, "latents_finite": finite,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
