"""world_size-2 and -4 gloo runs of the exact data-parallel code bench.py runs on the
8-GPU node (clap2diffusion_amd.distributed: env discovery, global-index sharding,
rank_inputs -- real synthetic audio, prompt selection, tokenize, per-sample seeded
initial_latents -- the timed loop with barrier + MAX-reduced timer, and the image
all-gather), with the GPU generation step replaced by a deterministic CPU stub.
Gathered latents and images must be bit-identical to one process generating every
sample (so the 1/2/4/8-GPU scaling runs generate the same images)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

PER_RANK = 2
HW = (8, 8)


def _stub_step(inp):
    """Stand-in for the GPU pipeline: a deterministic function of every per-sample input
    (waveform, prompt ids, latents) -> uint8 images [B, 8, 8, 3]."""
    a = torch.tensor([float(np.abs(x).mean()) for x in inp.audios])[:, None, None, None]
    t = (inp.ids_cond.sum(1) % 97).float()[:, None, None, None]
    u = (inp.ids_uncond.sum(1) % 13).float()[:, None, None, None]
    img = (inp.latents[:, :3] * 40 + 100 * a + t + u).abs().clamp(0, 255)
    return img.permute(0, 2, 3, 1).round().to(torch.uint8).contiguous()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from clap2diffusion_amd import distributed as D
    ctx = D.init("cpu")
    assert (ctx.rank, ctx.world, ctx.backend) == (rank, world, "gloo")
    inp = D.rank_inputs(ctx.shard(PER_RANK), HW, ctx.device)
    gathered = [torch.empty(PER_RANK, *HW, 3, dtype=torch.uint8) for _ in range(world)]

    def step():
        img = _stub_step(inp)
        ctx.all_gather(img, gathered)
        return img

    dt, last = D.timed_run(ctx, step, steps=2, warmup=1)
    lat = ctx.all_gather(inp.latents)
    mx = ctx.max_over_ranks(float(rank))
    if rank == 0:
        q.put((torch.cat(gathered).numpy(), torch.cat(lat).numpy(), mx, dt, inp.prompts))
    ctx.barrier()
    ctx.close()


@pytest.mark.parametrize("world,port", [(2, 29513), (4, 29517)])
def test_bench_dp_path_matches_one_process(world, port):
    from clap2diffusion_amd import distributed as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    imgs, lats, mx, dt, prompts0 = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    one = D.rank_inputs(list(range(PER_RANK * world)), HW, "cpu")   # single process, every sample
    assert (lats == one.latents.numpy()).all()
    assert (imgs == _stub_step(one).numpy()).all()
    assert mx == float(world - 1) and dt > 0
    assert prompts0 == [D.bench_prompt(i) for i in range(PER_RANK)]


def test_shard_and_seed_recipe():
    from clap2diffusion_amd import distributed as D
    assert D.shard_indices(8, 3) == list(range(24, 32))
    assert D.sample_seed(0, 5) == 5 and D.sample_seed(2, 5) == 2005
    ctx = D.DPContext()
    x = torch.arange(4)
    assert ctx.all_gather(x)[0] is x and ctx.max_over_ranks(1.5) == 1.5 and not ctx.distributed
