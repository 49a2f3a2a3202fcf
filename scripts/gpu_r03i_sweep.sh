#!/bin/bash
# Plan-table re-sweep after the fp16 split-K slabs: every UNet shape at c3 / c2 / c5 batches over
# the DMA tiles and split counts (graph-replayed; the 'default' column is the current plan).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for args in "--batch 8" "--batch 1" "--batch 4 --res 96"; do
  timeout -k 10 330 python -u scripts/sweep_tiles_graph.py $args --tiles 40,41,25,7,1,2,3,8,9 --splits 1,2,3,4,6,8,12,16 \
    --iters 10 || exit 1
done
