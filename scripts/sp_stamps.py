"""Per-K-step timeline of the software-pipelined GEMM (tile 60 / 61) from the diagnostic stamp build:
python -m clap2diffusion_amd.build --variant stamp --define C2D_SP_STAMP, then on the GPU
C2D_LIB=clap2diffusion_amd/libc2d_hip_stamp.so python scripts/sp_stamps.py --shape conv0 --tile 60
Prints, per wave of workgroup 77 (s_memtime cycles): prologue, per step groups 0-10, the vmcnt drain +
barrier X1, groups 11-13 + barrier X2, groups 14-15 + the next step's top wait, and the epilogue."""
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
PER = 6 * 64 + 4
buf = (ctypes.c_ulonglong * (8 * PER))()
assert _lib.lib().c2d_debug_sp_stamps(buf, 8 * PER) == 0
names = ["g0-10", "X1", "g11-13+X2", "g14", "g15", "top wait"]
for w in range(8):
    t = [buf[w * PER + i] for i in range(PER)]
    t0 = t[0]
    rows = []
    k = 0
    while 10 + 6 * (k + 1) < PER and t[4 + 6 * (k + 1)] > t0:
        b0 = 4 + 6 * k
        s_ = [t[b0 + j] for j in range(6)] + [t[b0 + 6]]
        rows.append([s_[j + 1] - s_[j] for j in range(6)])
        k += 1
    if not rows:
        continue
    med = [statistics.median(r[j] for r in rows) for j in range(6)]
    print(f"wave {w}: steps {len(rows) + 1}  prologue {t[1] - t0}  loop {t[2] - t[1]}  epilogue {t[3] - t[2]}  | per step: " +
          "  ".join(f"{n} {m:.0f}" for n, m in zip(names, med)) + f"  (sum {sum(med):.0f})")
