"""world_size-2 and -4 gloo runs of the data-parallel plumbing: sample sharding, per-sample
seeded latents identical to a single-process run, image all-gather (bit-identical images
for any rank count: the 1/2/4/8-GPU scaling runs generate the same samples)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from clap2diffusion_amd.distributed import gather_images, sample_seed, shard_indices


def _latents(indices):
    return torch.stack([torch.randn(4, 8, 8, generator=torch.Generator().manual_seed(sample_seed(0, i)))
                        for i in indices])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    idx = shard_indices(4, rank)
    lat = _latents(idx)
    img = (lat[:, :3].permute(0, 2, 3, 1).abs() * 50).clamp(0, 255).to(torch.uint8)  # stand-in images
    out = gather_images(img)
    if rank == 0:
        q.put(torch.cat(out).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,port", [(2, 29513), (4, 29517)])
def test_rank_shard_and_gather(world, port):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _latents(range(4 * world))
    ref_img = (ref[:, :3].permute(0, 2, 3, 1).abs() * 50).clamp(0, 255).to(torch.uint8).numpy()
    assert (got == ref_img).all()
