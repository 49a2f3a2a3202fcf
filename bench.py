#!/usr/bin/env python3
"""Benchmark: 512x512 images/sec @ 50 DDIM steps, batch 8 per GPU (BASELINE.json metric).

One bench "step" = one full generation of a batch of 8 images on every rank:
CLAP log-mel (HIP) -> HTSAT (HIP) -> audio projectors -> CLIP text tower -> 50 CFG+DDIM denoise steps of
the audio-conditioned SD1.5 UNet (HIP kernels) -> VAE decode -> RCCL all-gather of the uint8 images to
every rank; the conditioning leg, the denoise step and the VAE are hipGraphs (pipeline.BatchGraph).  Inputs (48 kHz waveforms,
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

PEAK_F16_TFLOPS = 2500.0  # MI355X dense fp16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
UNET_GFLOP_PER_SAMPLE = 803.2  # SURVEY.md Appendix C, 64x64 latent


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def measure_dominant_kernel(dev, iters: int = 20):
    """The dominant kernel is the implicit-GEMM conv (c2d_conv2d_igemm): time its
    most frequent heavy launch, the level-0 ResnetBlock2D conv2 (320 -> 320, 3x3 + residual,
    N = 16 CFG images, 64x64) as the UNet runs it -- over the zero-bordered GroupNorm output
    (c2d_groupnorm_pad) on the row-ring tile 42 -- with HIP events on the stream it is
    launched on."""
    from clap2diffusion_amd import ops
    n, h, c = 16, 64, 320
    x = torch.randn(n, h, h, c, device=dev, dtype=torch.float16)
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1)).contiguous()   # [n, h + 2, w + 2, c], zero border
    w = torch.randn(c, c, 3, 3, device=dev) / math.sqrt(9 * c)
    wp, kp = ops.pack_conv_weight(w)
    b = torch.zeros(c, device=dev)
    res = torch.randn_like(x)
    out = torch.empty_like(x)

    def call():
        ops.conv(xp, wp, kp, c, ksize=3, bias=b, resid=res, out=out, padded=True)
    with ops.record_conv_plans() as plans:
        call()
    for _ in range(2):
        call()
    tile, split = plans[0]
    kname = {42: "igemm_pp16r_kernel<5,4> 256x320 row-ring ping-pong 16x16x32 over the zero-bordered source",
             40: "igemm_pp16_kernel<5,3,4> 256x320 ping-pong 16x16x32, 4 phases per K step",
             25: "igemm_m32_kernel 256x320 32x32x16"}.get(tile, f"tile {tile}")
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        call()
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flop = 2.0 * n * h * h * c * (9 * c)
    tflops = flop / (ms * 1e-3) / 1e12
    return {"bound": "mfma", "achieved": round(tflops, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tflops / PEAK_F16_TFLOPS, 4), "traffic": None,
            "kernel": f"c2d_conv2d_igemm ({kname}, split {split}) level-0 ResnetBlock2D conv2 3x3 320->320 + "
                      "residual, N=16 (CFG pair x 8 images) x 64x64",
            "flop_per_launch": flop, "avg_us": round(ms * 1e3, 2)}


def family_fractions(den):
    """roofline.family_frac: per kernel family of one denoise step of the benchmarked batch, the
    family's algorithmic work over its time -- FLOP / (time x 2.5 PF/s) for the MFMA families,
    bytes / (time x 8 TB/s) for the HBM ones -- with every c2d call of the step recorded and each
    unique call timed as a graph of back-to-back replays (scripts/ledger.py, whose full per-shape
    table for c3 / c2 is profiles/r05_ledger_*.txt)."""
    sys.path.insert(0, str(ROOT / "scripts"))
    from ledger import PEAK_BYTES, PEAK_FLOPS, step_ledger
    rows, fams, meta = step_ledger(den, situ=True)
    out = {}
    for f, s in fams.items():
        out[f] = round(s["mfma_frac"] if s["flop"] > 0 else s["frac"], 4)
    step_ms = None if meta["step_us"] is None else meta["step_us"] / 1e3

    def frac_of(flop, byts, us):
        return round((flop / PEAK_FLOPS if flop > 0 else byts / PEAK_BYTES) * 1e6 / us, 4) if us > 0 else None
    si = meta["in_situ"]
    situ_frac = {f: frac_of(fams[f]["flop"], fams[f]["bytes"], us) for f, us in si["family_us"].items()}
    all_us = si["sequence_us"]
    situ_frac["all"] = frac_of(fams["all"]["flop"], 0.0, all_us)
    r, us = max(si["heavy"], key=lambda t: t[1])
    dom = {"kernel": f"{r['family']}: {r['desc']}", "plan": r["plan"], "calls_per_step": r["calls"],
           "ms_per_step_in_situ": round(us / 1e3, 3),
           "share_of_step": None if step_ms is None else round(us / 1e3 / step_ms, 4),
           "frac_in_situ": frac_of(r["calls"] * r["flop"], r["calls"] * r["bytes"], us),
           "us_per_call_isolated": round(r["us"], 1)}
    return out, {"ledger_ms_per_step": round(fams["all"]["us"] / 1e3, 3),
                 "step_graph_ms": None if step_ms is None else round(step_ms, 3),
                 "ledger_gap_ms": None if step_ms is None else round(step_ms - fams["all"]["us"] / 1e3, 3),
                 "family_ms_per_step": {f: round(s["us"] / 1e3, 3) for f, s in fams.items()},
                 "family_frac_in_situ": situ_frac,
                 "family_ms_in_situ": {f: round(u / 1e3, 3) for f, u in si["family_us"].items()},
                 "sequence_graph_ms": round(all_us / 1e3, 3),
                 "dominant_by_time": dom,
                 "in_situ_source": "scripts/ledger.py in_situ: the step's recorded c2d calls captured in order as one graph "
                                   "(sequence_graph_ms) and again without each family / heavy signature; a family's in-situ "
                                   "time is the difference, its frac = its FLOP (bytes) / (that time x 2.5 PF/s (8 TB/s)); "
                                   "all = every FLOP of the step over the sequence time",
                 "family_source": "scripts/ledger.py step_ledger: every c2d call of one denoise step, each unique "
                                  "call timed as a graph of 10 back-to-back replays; FLOP / (t x 2.5 PF/s) for "
                                  "families with FLOP, bytes / (t x 8 TB/s) for norms and elementwise"}


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


def cpu_baseline(cores: int | None = None):
    """Config c1 of BASELINE.json / BASELINE.md §2 on the host cores: the full fp32 CPU
    pipeline (oracle/pipeline_ref.py, the port of the diffusers + transformers path the
    reference glues together): preprocess + log-mel -> HTSAT -> projectors -> CLIP ->
    10 CFG+DDIM UNet calls at 512^2 (64^2 latent, N = 2) -> VAE decode, B = 1,
    synthetic "Thunder" clip + "a beach".  One timed run after a one-UNet-call warm-up
    (a median of 3 would take ~4 minutes); weights are built before the clock starts.
    The 50-step figure is extrapolated from the measured stage times."""
    from clap2diffusion_amd.distributed import sample_seed
    from clap2diffusion_amd.pipeline import initial_latents, synthetic_thunder
    from clap2diffusion_amd.text_encoder import tokenize
    from oracle.pipeline_ref import ReferencePipeline
    cores = cores or min(16, os.cpu_count() or 1)
    torch.set_num_threads(cores)
    ref = ReferencePipeline(0)
    lat = initial_latents([sample_seed(0, 0)], 64, 64)
    ids_u, ids_c = tokenize([""]), tokenize(["a beach"])
    with torch.no_grad():   # warm-up: one CFG-pair UNet call (oneDNN primitive creation)
        ref.unet(torch.cat([lat, lat]), 981, torch.zeros(2, 77, 768), None)
    tm = {}
    ref.run([synthetic_thunder(0)], ids_u, ids_c, lat, 10, 7.5, timings=tm)
    unet_call = float(np.median(tm["unet"]))
    fixed = tm["mel"] + tm["condition"] + tm["vae"]
    s50 = fixed + 50 * unet_call
    # value in the metric's unit (512^2 images/s at 50 DDIM steps): the measured fixed stages plus
    # 50 x the measured median CFG-pair UNet call; the measured 10-step c1 rate is its own field
    return {"value": round(1.0 / s50, 6), "unit": "images/sec (512^2, 50 DDIM steps)", "cores": cores,
            "kind": "port",
            "sample": f"config c1 measured (1 x 512^2, 10 DDIM steps, fp32 CPU pipeline: log-mel, HTSAT, projectors, "
                      f"CLIP, 10 CFG-pair UNet calls, VAE; {cores} threads, 1 run after warm-up), scaled to 50 steps "
                      f"with the measured per-call UNet time",
            "c1_seconds_per_image": round(tm["total"], 2),
            "c1_images_per_s_10_steps": round(1.0 / tm["total"], 6),
            "stage_seconds": {"mel": round(tm["mel"], 3), "condition": round(tm["condition"], 3),
                              "unet_call_median": round(unet_call, 3), "unet_total": round(sum(tm["unet"]), 2),
                              "vae": round(tm["vae"], 2)},
            "seconds_per_image_50_steps": round(s50, 2)}


def gpu_config_runs(pipe, dev, log):
    """The other single-GPU configs of BASELINE.json, measured in the same process after the
    headline run: c2 (B = 1, 50 steps, 512^2: latency, median of 5 after a warm-up), c1's
    workload on the GPU (B = 1, 10 steps), c5 (768^2, B = 4, 50 steps: images/s)."""
    from clap2diffusion_amd.distributed import rank_inputs

    def gen(b, res, steps, reps, warm):
        inp = rank_inputs(list(range(b)), (res // 8, res // 8), dev)
        clips = pipe.feature_extractor.crop(inp.audios)
        wave = torch.from_numpy(np.concatenate(clips)).to(dev)
        lens = torch.tensor([c.size for c in clips], dtype=torch.int32, device=dev)
        offs = torch.tensor(np.cumsum([0] + [c.size for c in clips[:-1]]), dtype=torch.int64, device=dev)

        def one():
            return pipe.generate_batch_graphed(wave, offs, lens, (inp.ids_uncond, inp.ids_cond), inp.latents, steps,
                                               7.5)
        for _ in range(warm):
            one()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            one()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return ts

    out = {}
    ts = gen(1, 512, 50, 5, 2)
    out["c2_latency_s"] = round(float(np.median(ts)), 4)
    log(f"[bench] c2 latency {out['c2_latency_s']} s")
    ts = gen(1, 512, 10, 5, 2)
    out["c1_gpu_latency_s"] = round(float(np.median(ts)), 4)
    ts = gen(4, 768, 50, 2, 1)
    out["c5_images_per_s"] = round(4 / float(np.mean(ts)), 4)
    log(f"[bench] c5 {out['c5_images_per_s']} img/s")
    return out


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
    ap.add_argument("--no-configs", action="store_true", help="skip the c1/c2/c5 side measurements")
    ap.add_argument("--dtype", default="fp16", choices=["fp16"],
                    help="compute dtype of the HIP path (fp16 storage, fp32 accumulation; the only one built)")
    a = ap.parse_args()

    from clap2diffusion_amd import distributed as D
    from clap2diffusion_amd.pipeline import AudioToImageInference

    ctx = D.init("cuda")
    dev = ctx.device
    t_setup = time.time()
    pipe = AudioToImageInference(device=dev, height=a.res, width=a.res, verbose=False)
    B = a.batch
    inp = D.rank_inputs(ctx.shard(B), (a.res // 8, a.res // 8), dev)
    # waveforms resident in HBM; the log-mel front end (c2d_clap_log_mel) runs inside the step
    clips = pipe.feature_extractor.crop(inp.audios)
    wave = torch.from_numpy(np.concatenate(clips)).to(dev)
    lens = torch.tensor([c.size for c in clips], dtype=torch.int32, device=dev)
    offs = torch.tensor(np.cumsum([0] + [c.size for c in clips[:-1]]), dtype=torch.int64, device=dev)
    gathered = [torch.empty(B, a.res, a.res, 3, dtype=torch.uint8, device=dev) for _ in range(ctx.world)]
    if ctx.rank == 0:
        log(f"[bench] setup {time.time() - t_setup:.1f}s, world={ctx.world}, batch/gpu={B}")

    def one_batch():
        # the whole batch as hipGraphs: conditioning leg, 50 denoise-step replays, VAE (BatchGraph)
        img = pipe.generate_batch_graphed(wave, offs, lens, (inp.ids_uncond, inp.ids_cond), inp.latents,
                                          a.ddim_steps, 7.5)
        ctx.all_gather(img, gathered)
        return img

    dt, _ = D.timed_run(ctx, one_batch, a.steps, a.warmup, torch.cuda.synchronize,
                        log=lambda m: log("[bench] " + m))
    finite = bool(torch.isfinite(pipe.last_denoiser.x).all().item())
    ms_per_step = dt / a.steps * 1e3
    total_images = ctx.world * B * a.steps
    value = total_images / dt

    if ctx.rank == 0:
        roof = measure_dominant_kernel(dev)
        unet_tf = UNET_GFLOP_PER_SAMPLE * (a.res / 512) ** 2 * 2 * a.ddim_steps * total_images / dt / 1e3
        roof["pipeline_unet_tflops"] = round(unet_tf, 2)
        n_, h_, c_ = 16, 64, 320
        # padded x + resid + out + weights
        roof["algorithmic_bytes"] = 2 * (n_ * (h_ + 2) ** 2 * c_ + 2 * n_ * h_ * h_ * c_ + c_ * 9 * c_)
        try:
            roof["family_frac"], fam_meta = family_fractions(pipe.last_denoiser)
            roof.update(fam_meta)
        except Exception as e:  # noqa: BLE001 - reported, never fatal to the bench
            roof["family_frac"], roof["family_source"] = None, f"ledger failed: {type(e).__name__}: {e}"
        if not a.no_pmc and ctx.world == 1:
            tr, src = pmc_traffic()
            roof["traffic"] = None if tr is None else round(tr)
            roof["traffic_source"] = src
        extra = {}
        if not a.no_configs and ctx.world == 1 and (a.res, B) == (512, 8):
            extra = gpu_config_runs(pipe, dev, log)
        cpu = None if (a.no_cpu_baseline or ctx.world > 1) else cpu_baseline()
        # BASELINE.json configs: c3 is the default line; other shapes are labelled, not the metric
        cfg_name = {(512, 8): "c3", (512, 1): "c2", (768, 4): "c5"}.get((a.res, B), "custom")
        if ctx.world > 1 and (a.res, B) == (512, 8):
            cfg_name = "c4" if ctx.world == 8 else "c3-sharded"
        line = {
            "metric": "512x512 images/sec @ 50 DDIM steps, batch=8, 1/2/4/8 MI355X",
            "value": round(value, 4), "unit": "images/sec", "n_gpus": ctx.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic (seeded thunder-like audio, fixed token ids, random-init SD1.5/CLAP weights)",
            "config": {"workload": f"{cfg_name}: batch={B}/GPU, {a.ddim_steps} DDIM steps, {a.res}x{a.res}, CFG 7.5, "
                                   "log-mel+HTSAT+projectors+CLIP+UNet+VAE, all-gather of images",
                       "global_batch": B * ctx.world, "ddim_steps": a.ddim_steps, "resolution": a.res,
                       "parallelism": f"dp{ctx.world}"},
            "roofline": roof, "cpu_baseline": cpu, "latents_finite": finite, **extra,
        }
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
