"""End-to-end fp32 CPU reference of the sampling path (TEST ORACLE ONLY):
waveform -> preprocess + log-mel (mel_ref) -> HTSAT (htsat_ref) -> the projectors' routed
tokens (projectors_ref: plain tensor functions, pinned by tests/golden/projectors.npz; the
product's projector modules are not used here) -> CLIP text tower (transformers CLIPTextModel,
clip_ref) -> UNetRef + DDIM/CFG (ddim_ref) -> VAEDecoderRef, on the same seeded
weights as clap2diffusion_amd.pipeline.AudioToImageInference(seed).

Also the CPU leg of bench.py (config c1 of BASELINE.json: 1 x 512^2, 10 DDIM
steps, fp32, "Thunder" + "a beach"), so every stage is timed separately."""
from __future__ import annotations

import time

import numpy as np
import torch

from clap2diffusion_amd import weights as W
from oracle.clip_ref import clip_text_model
from oracle.ddim_ref import alphas_cumprod, ddim_step, timesteps
from oracle.htsat_ref import htsat_forward
from oracle.mel_ref import log_mel
from oracle.projectors_ref import projector_shapes, routed_tokens
from oracle.unet_ref import UNetRef
from oracle.vae_ref import VAEDecoderRef


class ReferencePipeline:
    """All weights built once (model load is not part of any timing)."""

    def __init__(self, seed: int = 0):
        self.seed = seed
        self.htsat_sd = W.synth_htsat(seed)
        # the product's seeded recipe, key by key (W.synth_generic seeds every tensor from its name):
        # the same projector weights as pipeline.AudioToImageInference(seed), without its modules
        self.enc_sd = W.synth_generic(projector_shapes(), seed, "improved.")
        self.clip = clip_text_model(seed)
        procs = {lv: W.synth_processor_weights(lv, seed) for lv in ("early", "mid", "late")}
        self.unet = UNetRef(W.synth_unet(seed), processors=procs)
        self.vae = VAEDecoderRef(W.synth_vae_decoder(seed))

    @torch.no_grad()
    def mel(self, waves: list) -> torch.Tensor:
        """48 kHz clips -> [B, 1001, 64] fp32 (reference preprocess_audio + extractor)."""
        return torch.from_numpy(np.stack([log_mel(w) for w in waves]).astype(np.float32))

    @torch.no_grad()
    def condition(self, mel: torch.Tensor, ids_uncond: torch.Tensor, ids_cond: torch.Tensor):
        clap = htsat_forward(self.htsat_sd, mel[:, None].float())
        audio = {k: torch.cat([v, v], 0) for k, v in routed_tokens(clap, self.enc_sd)["routed"].items()}
        ehs = self.clip(input_ids=torch.cat([ids_uncond, ids_cond], 0).cpu()).last_hidden_state.float()
        return ehs, audio

    @torch.no_grad()
    def run(self, mel_or_waves, ids_uncond: torch.Tensor, ids_cond: torch.Tensor, latents: torch.Tensor,
            steps: int, guidance: float = 7.5, timings: dict | None = None, progress=None):
        """-> (uint8 NHWC images, final latents).  timings (optional dict) receives the
        seconds spent per stage: mel, condition, unet (list, one per CFG-pair call), vae;
        progress (optional callable) gets a short string after every UNet call."""
        tm = timings if timings is not None else {}
        t0 = time.perf_counter()
        mel = mel_or_waves if isinstance(mel_or_waves, torch.Tensor) else self.mel(mel_or_waves)
        t1 = time.perf_counter()
        ehs, audio = self.condition(mel.cpu(), ids_uncond, ids_cond)
        t2 = time.perf_counter()
        ac = alphas_cumprod()
        x = latents.float().cpu().clone()
        tm["unet"] = []
        for t in timesteps(steps):
            ts = time.perf_counter()
            eps = self.unet(torch.cat([x, x], 0), int(t), ehs, audio)
            eu, ec = eps.chunk(2)
            x = ddim_step(eu + guidance * (ec - eu), int(t), x, steps, ac)
            tm["unet"].append(time.perf_counter() - ts)
            if progress is not None:
                progress(f"oracle step {len(tm['unet'])}/{steps} t={int(t)} {tm['unet'][-1]:.1f}s")
        t3 = time.perf_counter()
        img = self.vae(x)
        t4 = time.perf_counter()
        tm.update(mel=t1 - t0, condition=t2 - t1, vae=t4 - t3, total=t4 - t0)
        return (img.permute(0, 2, 3, 1) * 255).round().to(torch.uint8), x


@torch.no_grad()
def reference_images(mel: torch.Tensor, ids_uncond: torch.Tensor, ids_cond: torch.Tensor, latents: torch.Tensor,
                     steps: int, guidance: float = 7.5, seed: int = 0):
    """-> (uint8 NHWC images (CPU), final latents)."""
    return ReferencePipeline(seed).run(mel, ids_uncond, ids_cond, latents, steps, guidance)
