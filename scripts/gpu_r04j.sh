#!/bin/bash
# Round 4: graph-replayed (tile, split-K) re-sweep of the UNet shapes with fp32 split-K slabs
# (the round-3 plan table was tuned with fp16 slabs): c3 (batch 8) split-able shapes, c2 (batch 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 400 python -u scripts/sweep_tiles_graph.py --batch 8 --only "L2" --splits 1,2,3,4,6,8 > $O/sweep_b8_l2.txt 2>&1 || { tail -5 $O/sweep_b8_l2.txt; exit 1; }
timeout -k 10 400 python -u scripts/sweep_tiles_graph.py --batch 8 --only "L3" --splits 1,2,4,6,8,12,16 > $O/sweep_b8_l3.txt 2>&1 || { tail -5 $O/sweep_b8_l3.txt; exit 1; }
timeout -k 10 400 python -u scripts/sweep_tiles_graph.py --batch 8 --only "L1 3x3" --splits 1,2,3,4 > $O/sweep_b8_l1.txt 2>&1 || { tail -5 $O/sweep_b8_l1.txt; exit 1; }
timeout -k 10 500 python -u scripts/sweep_tiles_graph.py --batch 1 --only "3x3" --splits 1,2,4,6,8,12,16 > $O/sweep_b1_3x3.txt 2>&1 || { tail -5 $O/sweep_b1_3x3.txt; exit 1; }
echo sweeps done
