"""DDIM (eta = 0) + classifier-free guidance, fp32 CPU (TEST ORACLE ONLY).

Restates diffusers==0.23.1 DDIMScheduler with the SD1.5 scheduler config
(SURVEY.md Appendix A): num_train_timesteps 1000, scaled_linear betas
0.00085 -> 0.012, set_alpha_to_one False, steps_offset 1, timestep_spacing
"leading", prediction_type epsilon, clip_sample False; and the pipeline's CFG
combine eps = eps_u + g (eps_c - eps_u) with the [uncond, cond] batch order.
Reference defaults: 50 steps, guidance 7.5 (scripts/inference.py:106-107).
"""
from __future__ import annotations

import numpy as np
import torch


def alphas_cumprod(n_train: int = 1000, beta_start: float = 0.00085, beta_end: float = 0.012) -> torch.Tensor:
    betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, n_train, dtype=torch.float32) ** 2
    return torch.cumprod(1.0 - betas, dim=0)


def timesteps(num_steps: int, n_train: int = 1000, offset: int = 1) -> np.ndarray:
    ratio = n_train // num_steps
    t = (np.arange(0, num_steps) * ratio).round()[::-1].copy().astype(np.int64)
    return t + offset


def ddim_step(eps: torch.Tensor, t: int, x: torch.Tensor, num_steps: int, ac: torch.Tensor) -> torch.Tensor:
    prev = t - 1000 // num_steps
    a_t = ac[t]
    a_p = ac[prev] if prev >= 0 else ac[0]
    x0 = (x - (1 - a_t) ** 0.5 * eps) / a_t ** 0.5
    return a_p ** 0.5 * x0 + (1 - a_p) ** 0.5 * eps


def sample(unet, latents: torch.Tensor, ehs: torch.Tensor, audio: dict | None, num_steps: int,
           guidance: float = 7.5) -> torch.Tensor:
    """latents [B,4,h,w]; ehs [2B,77,768] ordered [uncond, cond]; audio {level: [2B,K,768]}."""
    ac = alphas_cumprod()
    x = latents.float().clone()
    for t in timesteps(num_steps):
        inp = torch.cat([x, x], dim=0)
        eps = unet(inp, int(t), ehs, audio)
        eu, ec = eps.chunk(2)
        e = eu + guidance * (ec - eu)
        x = ddim_step(e, int(t), x, num_steps, ac)
    return x
