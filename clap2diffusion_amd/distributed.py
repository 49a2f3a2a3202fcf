"""Data parallelism over independent samples.

One process per GPU (torch.distributed.run: RANK / WORLD_SIZE / LOCAL_RANK /
MASTER_* in the environment); rank r of g owns the global samples
[r*B, (r+1)*B) of a batch of g*B; every sample's CFG pair stays on its rank.
Per-sample inputs (waveform seed, prompt, initial-latent seed) are functions of
the GLOBAL sample index only, so 1/2/4/8-GPU runs generate bit-identical
images.  The only data-path collective is the end-of-batch all-gather of the
finished uint8 images (RCCL over xGMI with backend "nccl" on ROCm; gloo in the
CPU tests); the timer is reduced with one MAX all-reduce after the timed region.

This module is the code bench.py runs on the 8-GPU node, and the code
tests/test_distributed_cpu.py drives under gloo at world sizes 2 and 4 with the
GPU step stubbed out.  The reference has no multi-GPU path.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch
import torch.distributed as dist

# prompts of the synthetic workload (fixed token ids; no tokenizer offline)
BENCH_PROMPTS = ("a beach", "a city street at night")


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def shard_indices(per_rank: int, rank: int) -> list[int]:
    """Global sample indices of `rank` when every rank owns `per_rank` consecutive samples."""
    return [rank * per_rank + i for i in range(per_rank)]


def sample_seed(base_seed: int, global_index: int) -> int:
    """Initial-latent seed of a global sample (AudioToImageInference.batch_generate's recipe)."""
    return base_seed * 1000 + global_index


def bench_prompt(global_index: int) -> str:
    return BENCH_PROMPTS[global_index % len(BENCH_PROMPTS)]


@dataclass
class DPContext:
    """Rank / world of this process and the collectives the sampling path uses."""
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: str | None = None

    @property
    def distributed(self) -> bool:
        return self.world > 1

    def shard(self, per_rank: int) -> list[int]:
        return shard_indices(per_rank, self.rank)

    def barrier(self) -> None:
        if self.distributed:
            dist.barrier()

    def all_gather(self, t: torch.Tensor, out: list[torch.Tensor] | None = None) -> list[torch.Tensor]:
        """All-gather a per-rank tensor (same shape everywhere), rank order."""
        if not self.distributed:
            return [t]
        if out is None:
            out = [torch.empty_like(t) for _ in range(self.world)]
        if self.backend == "gloo" and t.is_cuda:   # rehearsal path: gloo gathers host copies
            host = [torch.empty_like(t, device="cpu") for _ in range(self.world)]
            dist.all_gather(host, t.contiguous().cpu())
            for o, h in zip(out, host):
                o.copy_(h)
            return out
        dist.all_gather(out, t.contiguous())
        return out

    def max_over_ranks(self, x: float) -> float:
        if not self.distributed:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def close(self) -> None:
        if self.distributed and dist.is_initialized():
            dist.destroy_process_group()


def init(device_type: str = "cuda", backend: str | None = None) -> DPContext:
    """Read the launcher environment; for world > 1 bind this process to its GPU
    (LOCAL_RANK) and join the process group ("nccl" = RCCL for cuda, "gloo" for cpu).
    Rehearsal knobs (a one-GPU box running several ranks): C2D_DP_ONE_DEVICE=1 puts every
    rank on cuda:0, C2D_DP_BACKEND=gloo replaces RCCL (which needs one GPU per rank)."""
    rank, ws, local = world()
    if device_type == "cuda":
        dev = torch.device("cuda", 0 if os.environ.get("C2D_DP_ONE_DEVICE") == "1" else local)
        if ws > 1:
            torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    be = backend or os.environ.get("C2D_DP_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if ws > 1 and not dist.is_initialized():
        if be == "nccl":
            dist.init_process_group(be, device_id=dev)
        else:
            dist.init_process_group(be, rank=rank, world_size=ws)
    return DPContext(rank, ws, local, dev, be if ws > 1 else None)


@dataclass
class RankInputs:
    """Host-side inputs of this rank's samples (all derived from global indices)."""
    indices: list[int]
    audios: list[np.ndarray]          # 48 kHz waveforms
    prompts: list[str]
    ids_uncond: torch.Tensor          # [B, 77] token ids of "" (CFG uncond half)
    ids_cond: torch.Tensor            # [B, 77] token ids of the prompts
    latents: torch.Tensor             # [B, 4, h, w] fp32, per-sample seeded


def rank_inputs(indices: list[int], latent_hw: tuple[int, int], device, base_seed: int = 0,
                audio_fn: Callable[[int], np.ndarray] | None = None) -> RankInputs:
    """The synthetic workload of SURVEY.md §8(d) for the given global sample indices:
    audio = synthetic_thunder(i), prompt = bench_prompt(i), latent seed = sample_seed(0, i)."""
    from .pipeline import initial_latents, synthetic_thunder
    from .text_encoder import tokenize
    audio_fn = audio_fn or synthetic_thunder
    prompts = [bench_prompt(i) for i in indices]
    return RankInputs(
        indices=list(indices),
        audios=[audio_fn(i) for i in indices],
        prompts=prompts,
        ids_uncond=tokenize([""] * len(indices), device),
        ids_cond=tokenize(prompts, device),
        latents=initial_latents([sample_seed(base_seed, i) for i in indices], *latent_hw, device=device),
    )


def timed_run(ctx: DPContext, step: Callable[[], object], steps: int, warmup: int,
              sync: Callable[[], None] = lambda: None, log: Callable[[str], None] | None = None):
    """warmup untimed steps, then exactly `steps` steps bracketed by a barrier and a device
    sync on both sides; returns (max-over-ranks seconds, last step output)."""
    out = None
    for i in range(warmup):
        out = step()
        sync()
        if log is not None and ctx.rank == 0:
            log(f"warmup {i} done")
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    ctx.barrier()
    dt = time.perf_counter() - t0
    return ctx.max_over_ranks(dt), out


def gather_images(img: torch.Tensor, out: list[torch.Tensor] | None = None) -> list[torch.Tensor]:
    """All-gather [B, H, W, 3] uint8 images from every rank (rank order) in the default group."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return [img]
    ws = dist.get_world_size()
    if out is None:
        out = [torch.empty_like(img) for _ in range(ws)]
    dist.all_gather(out, img.contiguous())
    return out
