#!/bin/bash
# Split-K 12 / 16 for the c2 (N = 2) small-M convs; GEGLU tiles at the three batches (tile 41 now runs
# two phases per K step on 1x1 shapes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/sw2
s() { timeout -k 10 300 python -u scripts/sweep_tiles_graph.py "$@" 2>&1 | grep " us " || exit 1; }
echo "== b1 L3"; s --batch 1 --only "L3" --tiles 3,9,2,7,8,41 --splits 4,6,8,12,16
echo "== b1 L2 3x3"; s --batch 1 --only "L2 3x3" --tiles 3,9,7,8,41 --splits 6,8,12,16
echo "== b1 L1 3x3"; s --batch 1 --only "L1 3x3" --tiles 3,9,7,8,41 --splits 6,8,12,16
echo "== b8 geglu"; s --batch 8 --only "geglu" --tiles 25,41,50,1 --splits 1
echo "== b4r96 geglu"; s --batch 4 --res 96 --only "geglu" --tiles 25,41,50,1 --splits 1
echo "== b1 geglu"; s --batch 1 --only "geglu" --tiles 25,41,50,1,3 --splits 1
