#!/bin/bash
# Round 4: per-shape breakdown of one c3 UNet call (N = 16, 64^2) and one c2 call (N = 2) on the
# current tree; then the by-kernel trace of one c3 batch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 300 python -u scripts/unet_shapes.py --batch 8 > $O/shapes_b8.txt 2>&1 || { tail -5 $O/shapes_b8.txt; exit 1; }
grep -v amdgpu.ids $O/shapes_b8.txt | head -70
timeout -k 10 300 python -u scripts/unet_shapes.py --batch 1 > $O/shapes_b1.txt 2>&1 || { tail -5 $O/shapes_b1.txt; exit 1; }
grep -v amdgpu.ids $O/shapes_b1.txt | head -40
