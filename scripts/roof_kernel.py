"""Run only bench.py's dominant kernel (the level-0 ResnetBlock2D conv, implicit GEMM
320->320 3x3 at N=16, 64x64) so rocprofv3 --pmc passes see exactly that launch.
python scripts/roof_kernel.py [iters]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import bench  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
r = bench.measure_dominant_kernel(torch.device("cuda:0"), iters=iters)
print(r, flush=True)
