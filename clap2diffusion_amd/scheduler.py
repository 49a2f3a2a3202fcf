"""DDIM scheduler (diffusers 0.23.1 DDIMScheduler semantics, SD1.5 config).

scaled_linear betas 0.00085 -> 0.012 over 1000 train steps, set_alpha_to_one
False (final alpha_cumprod = alphas_cumprod[0]), steps_offset 1, "leading"
timestep spacing, eta 0, epsilon prediction, no clipping.  Besides the
diffusers-style set_timesteps / step API (torch, host-driven), `device_tables`
returns the per-step (timestep, alpha_t, alpha_prev) tables the fused
c2d_cfg_ddim_step kernel reads through a device step counter, so a captured
hipGraph of one denoise step can be replayed for every step.
"""
from __future__ import annotations

import numpy as np
import torch


class DDIMScheduler:
    def __init__(self, num_train_timesteps: int = 1000, beta_start: float = 0.00085, beta_end: float = 0.012,
                 steps_offset: int = 1, set_alpha_to_one: bool = False):
        self.num_train_timesteps = num_train_timesteps
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        self.alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.steps_offset = steps_offset
        self.init_noise_sigma = 1.0
        self.num_inference_steps = None
        self.timesteps = None

    def set_timesteps(self, num_inference_steps: int, device=None) -> None:
        ratio = self.num_train_timesteps // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64) + self.steps_offset
        self.num_inference_steps = num_inference_steps
        self.timesteps = torch.from_numpy(ts).to(device) if device is not None else torch.from_numpy(ts)

    def scale_model_input(self, sample, timestep=None):
        return sample

    def _alphas(self, t: int):
        prev = t - self.num_train_timesteps // self.num_inference_steps
        a_t = self.alphas_cumprod[t]
        a_p = self.alphas_cumprod[prev] if prev >= 0 else self.final_alpha_cumprod
        return a_t, a_p

    def step(self, model_output: torch.Tensor, timestep: int, sample: torch.Tensor):
        a_t, a_p = self._alphas(int(timestep))
        x0 = (sample - (1 - a_t) ** 0.5 * model_output) / a_t ** 0.5
        prev = a_p ** 0.5 * x0 + (1 - a_p) ** 0.5 * model_output
        return type("DDIMOutput", (), {"prev_sample": prev, "pred_original_sample": x0})()

    def device_tables(self, device) -> tuple[torch.Tensor, torch.Tensor]:
        """-> (t_table fp32 [S], coef fp32 [S, 2] = (alpha_t, alpha_prev))."""
        assert self.timesteps is not None, "call set_timesteps first"
        ts = [int(t) for t in self.timesteps]
        coef = torch.tensor([[float(a) for a in self._alphas(t)] for t in ts], dtype=torch.float32)
        return (torch.tensor(ts, dtype=torch.float32, device=device), coef.to(device))
