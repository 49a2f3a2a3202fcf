#!/bin/bash
# Round 4: graph-replayed (tile, split-K) sweep of c2's (N = 2) 1x1 / QKV / GEGLU / folded-ff shapes with the
# fp32 split-K slabs (the 3x3 shapes were re-swept in r04j)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ab; mkdir -p $O
for f in "1x1" "qkv" "geglu" "fold"; do
  timeout -k 10 280 python -u scripts/sweep_tiles_graph.py --batch 1 --only "$f" --splits 1,2,3,4,6,8,12,16 > $O/sweep_b1_$f.txt 2>&1 || { tail -5 $O/sweep_b1_$f.txt; exit 1; }
  grep -v amdgpu $O/sweep_b1_$f.txt | cut -c1-170
done
