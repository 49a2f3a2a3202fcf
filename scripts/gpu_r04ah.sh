#!/bin/bash
# Round 4: c5 (N = 8, 96^2 latents) graph-replayed (tile, split-K) re-sweep with the fp32 split-K slabs, every
# shape class (round 3 swept with fp16 slabs, profiles/r03_sweep_b4r96.txt)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ah; mkdir -p $O
for f in "L0" "L1" "L2" "L3"; do
  timeout -k 10 280 python -u scripts/sweep_tiles_graph.py --batch 4 --res 96 --only "$f" --splits 1,2,3,4,6,8,12 > $O/sweep_c5_$f.txt 2>&1 || { tail -5 $O/sweep_c5_$f.txt; exit 1; }
  grep -v amdgpu $O/sweep_c5_$f.txt | cut -c1-175
done
