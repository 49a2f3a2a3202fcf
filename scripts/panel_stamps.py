"""Per-block timeline of the panel GEMM (tile 70, K = 320 LDS-weight form) from the diagnostic stamp
build: python -m clap2diffusion_amd.build --variant pstamp --define C2D_PANEL_STAMP, then on the GPU
C2D_LIB=clap2diffusion_amd/libc2d_hip_pstamp.so python scripts/panel_stamps.py --shape geglu0
Prints per wave of workgroup 77 (s_memtime cycles): the panel load, and per column block (median over
blocks) the wait at each K step start, each K step, and the epilogue."""
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
ap.add_argument("--shape", default="geglu0")
a = ap.parse_args()
dev = torch.device("cuda")
c = ab_tiles.make(*ab_tiles.SHAPES[a.shape][:7], dev, *ab_tiles.SHAPES[a.shape][7:])
with ops.force_plan(70, 0):
    for _ in range(20):
        ab_tiles.call(c)
torch.cuda.synchronize()
PER = 2 + 8 * 16
buf = (ctypes.c_ulonglong * (8 * PER))()
assert _lib.lib().c2d_debug_panel_stamps(buf, 8 * PER) == 0
for w in range(8):
    t = [buf[w * PER + i] for i in range(PER)]
    t0 = t[0]
    blocks = []
    for b in range(16):
        s_ = t[2 + 8 * b: 10 + 8 * b]
        if s_[0] <= t0 or any(x < s_[0] for x in s_):
            break
        # start -> step-0 wait done, step t -> t + 1 (5 steps incl. its wait), loop end -> epilogue end
        blocks.append([s_[1] - s_[0]] + [s_[i + 1] - s_[i] for i in range(1, 6)] + [s_[7] - s_[6]] +
                      ([t[2 + 8 * (b + 1)] - s_[7]] if b + 1 < 16 and t[2 + 8 * (b + 1)] > s_[7] else [0]))
    if not blocks:
        continue
    med = [statistics.median(r[j] for r in blocks) for j in range(8)]
    print(f"wave {w}: panel load {t[1] - t0}  blocks {len(blocks)}  per block: wait0 {med[0]:.0f}  steps " +
          " ".join(f"{m:.0f}" for m in med[1:6]) + f"  epilogue {med[6]:.0f}  gap {med[7]:.0f}  "
          f"(block total {sum(med[:7]):.0f})")
