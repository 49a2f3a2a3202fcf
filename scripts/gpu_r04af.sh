#!/bin/bash
# Round 4: partial blocks per image on the two-launch GroupNorm path (C2D_GN_FOLD_CAP; C2D_GN_BLOCKS = blocks
# targeted per launch), per-call graph timing at N = 2 and N = 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for cap in 32 64 128 256; do
  echo "== N=2 C2D_GN_FOLD_CAP=$cap"
  GN_N=2 C2D_GN_FOLD_CAP=$cap timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep -v amdgpu | head -7 || exit 1
done
for nb in 512 1024 2048; do
  echo "== N=16 C2D_GN_FOLD_CAP=256 C2D_GN_BLOCKS=$nb"
  GN_N=16 C2D_GN_FOLD_CAP=256 C2D_GN_BLOCKS=$nb timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep -v amdgpu | head -7 || exit 1
done
