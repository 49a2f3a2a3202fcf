#!/bin/bash
# GroupNorm partial-block count A/B (C2D_GN_BLOCKS) on the UNet GN shapes, graph-replayed.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do
for b in 1024 512 2048 256; do
  echo "== C2D_GN_BLOCKS=$b"
  C2D_GN_BLOCKS=$b C2D_GN_FUSED_HW=256 timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep "^GN" || exit 1
done
done
