"""Per-K-step timeline of the software-pipelined GEMM (tile 60 / 61) from the diagnostic stamp build:
python -m clap2diffusion_amd.build --variant stamp --define C2D_SP_STAMP, then on the GPU
C2D_LIB=clap2diffusion_amd/libc2d_hip_stamp.so python scripts/sp_stamps.py --shape conv0 --tile 60
Prints, per wave of workgroup 77 (s_memtime cycles): prologue, per-step compute (group 0 -> 13),
the vmcnt / lgkmcnt drain before the barrier, the barrier wait, and the epilogue."""
import argparse
import ctypes
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import _lib, ops  # noqa: E402
sys.path.insert(0, str(Path(__file__).resolve().parent))
import ab_tiles  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="conv0")
ap.add_argument("--tile", type=int, default=60)
ap.add_argument("--split", type=int, default=0)
a = ap.parse_args()
dev = torch.device("cuda")
c = ab_tiles.make(*ab_tiles.SHAPES[a.shape][:7], dev, *ab_tiles.SHAPES[a.shape][7:])
with ops.force_plan(a.tile, a.split):
    for _ in range(20):
        ab_tiles.call(c)
torch.cuda.synchronize()
PER = 4 * 64 + 4
buf = (ctypes.c_ulonglong * (8 * PER))()
assert _lib.lib().c2d_debug_sp_stamps(buf, 8 * PER) == 0
for w in range(8):
    t = [buf[w * PER + i] for i in range(PER)]
    t0 = t[0]
    steps = []
    k = 0
    while 7 + 4 * k < PER and t[7 + 4 * k] > t0:
        s0, s1, s2, s3 = t[4 + 4 * k], t[5 + 4 * k], t[6 + 4 * k], t[7 + 4 * k]
        steps.append((s1 - s0, s2 - s1, s3 - s2))
        k += 1
    if not steps:
        continue
    nxt = [t[4 + 4 * (i + 1)] - t[7 + 4 * i] for i in range(len(steps) - 1)]
    comp = [x[0] for x in steps]
    drain = [x[1] for x in steps]
    bar = [x[2] for x in steps]
    print(f"wave {w}: steps {len(steps)}  prologue {t[1] - t0}  loop {t[2] - t[1]}  epilogue {t[3] - t[2]}  | per step: "
          f"g0-13 {statistics.median(comp):.0f}  drain {statistics.median(drain):.0f}  barrier {statistics.median(bar):.0f}  "
          f"g14-15 {statistics.median(nxt) if nxt else 0:.0f}  (max g0-13 {max(comp)}, max barrier {max(bar)})")
