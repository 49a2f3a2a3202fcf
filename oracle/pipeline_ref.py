"""End-to-end fp32 CPU reference of the sampling path (TEST ORACLE ONLY):
mel -> HTSAT (htsat_ref) -> ImprovedHierarchicalAudioEncoder (the API-kept
torch module, pinned by tests/golden/projectors.npz) -> CLIP text tower (fp32)
-> UNetRef + DDIM/CFG (ddim_ref) -> VAEDecoderRef, on the same seeded weights
as clap2diffusion_amd.pipeline.AudioToImageInference(seed)."""
from __future__ import annotations

import torch

from clap2diffusion_amd import weights as W
from clap2diffusion_amd.projectors import ImprovedHierarchicalAudioEncoder
from clap2diffusion_amd.text_encoder import clip_text_model
from oracle.ddim_ref import sample
from oracle.htsat_ref import htsat_forward
from oracle.unet_ref import UNetRef
from oracle.vae_ref import VAEDecoderRef


@torch.no_grad()
def reference_images(mel: torch.Tensor, ids_uncond: torch.Tensor, ids_cond: torch.Tensor, latents: torch.Tensor,
                     steps: int, guidance: float = 7.5, seed: int = 0) -> torch.Tensor:
    """-> uint8 NHWC images (CPU)."""
    clap = htsat_forward(W.synth_htsat(seed), mel[:, None].float())
    enc = W.fill_module(ImprovedHierarchicalAudioEncoder(), "improved.", seed).eval()
    _, info = enc(clap, return_all=True)
    audio = {k: torch.cat([v, v], 0) for k, v in info["routed"].items()}
    ehs = clip_text_model(seed)(input_ids=torch.cat([ids_uncond, ids_cond], 0).cpu()).last_hidden_state.float()
    procs = {lv: W.synth_processor_weights(lv, seed) for lv in ("early", "mid", "late")}
    unet = UNetRef(W.synth_unet(seed), processors=procs)
    x = sample(unet, latents.float().cpu(), ehs, audio, steps, guidance)
    img = VAEDecoderRef(W.synth_vae_decoder(seed))(x)
    return (img.permute(0, 2, 3, 1) * 255).round().to(torch.uint8), x
