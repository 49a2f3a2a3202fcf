"""CFG + DDIM denoise loop driven by a captured hipGraph.

One denoise step = latent -> NHWC fp16 (duplicated for the [uncond, cond]
CFG pair), sinusoidal timestep embedding, the HIP UNet forward, and the fused
CFG+DDIM update, which also advances a device-side step counter.  The step
reads its timestep and DDIM coefficients through that counter, so the same
graph is replayed for every step: no host work and no host<->device traffic
inside the 50-step loop.
"""
from __future__ import annotations

import torch

from . import ops
from .scheduler import DDIMScheduler


class GraphDenoiser:
    def __init__(self, unet, scheduler: DDIMScheduler, batch: int, height: int, width: int, guidance: float,
                 encoder_hidden_states: torch.Tensor, cross_attention_kwargs: dict | None, use_graph: bool = True):
        dev = encoder_hidden_states.device
        self.unet, self.sched = unet, scheduler
        self.b, self.h, self.w, self.g = batch, height, width, float(guidance)
        assert encoder_hidden_states.shape[0] == 2 * batch, "ehs must be [uncond; cond] for the CFG pair"
        self.ehs = encoder_hidden_states.to(torch.float16).contiguous()
        self.kw = cross_attention_kwargs or {}
        self.t_table, self.coef = scheduler.device_tables(dev)
        self.steps = self.t_table.numel()
        self.x = torch.zeros(batch, 4, height, width, dtype=torch.float32, device=dev)
        self.step_idx = torch.zeros(1, dtype=torch.int32, device=dev)
        self.use_graph = use_graph
        self.graph = None
        self.temb_ch = unet.cfg["block_out_channels"][0]

    def _body(self) -> None:
        xin = ops.latent_to_nhwc(self.x, self.unet.in_pad, dup=True)
        t_sin = ops.timestep_embedding(self.t_table, self.step_idx, 2 * self.b, self.temb_ch)
        eps = self.unet.forward_nhwc(xin, t_sin, self.ehs, self.kw)
        ops.cfg_ddim_step(eps, self.x, self.g, self.coef, self.step_idx, advance=True)

    def capture(self) -> None:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._body()  # warm-up: packs lazily-built weights, primes the allocator
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._body()
        self.step_idx.zero_()

    @torch.no_grad()
    def run(self, latents: torch.Tensor) -> torch.Tensor:
        """latents [B,4,h,w] (scaled by init_noise_sigma = 1) -> denoised latents fp32."""
        if self.use_graph and self.graph is None:
            self.capture()
        self.x.copy_(latents)
        self.step_idx.zero_()
        for _ in range(self.steps):
            if self.use_graph:
                self.graph.replay()
            else:
                self._body()
        return self.x
