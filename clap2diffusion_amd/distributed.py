"""Data parallelism over independent samples.

One process per GPU; rank r of g owns global samples [r*B, (r+1)*B) of a
batch of g*B; every sample's CFG pair stays on its rank; initial latents come
from a per-sample CPU generator, so 1/2/4/8-GPU runs produce identical images.
The only collective is the end-of-batch all-gather of the finished uint8
images (RCCL over xGMI with backend "nccl" on ROCm; gloo in the CPU tests).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def shard_indices(per_rank: int, rank: int) -> list[int]:
    return [rank * per_rank + i for i in range(per_rank)]


def sample_seed(base_seed: int, global_index: int) -> int:
    return base_seed * 1000 + global_index


def gather_images(img: torch.Tensor, out: list[torch.Tensor] | None = None) -> list[torch.Tensor]:
    """All-gather [B, H, W, 3] uint8 images from every rank (rank order)."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return [img]
    ws = dist.get_world_size()
    if out is None:
        out = [torch.empty_like(img) for _ in range(ws)]
    dist.all_gather(out, img.contiguous())
    return out
