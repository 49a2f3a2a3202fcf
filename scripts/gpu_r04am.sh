#!/bin/bash
# Round 4: apply workgroups per launch on the two-launch GroupNorm path (C2D_GN_APPLY_BLOCKS: every apply
# workgroup folds its image's group pairs first), per-call graph timing at N = 2 and N = 16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for n in 2 16; do for ab in 256 512 1024 2048; do
  echo "== N=$n C2D_GN_APPLY_BLOCKS=$ab"
  GN_N=$n C2D_GN_APPLY_BLOCKS=$ab timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep -v amdgpu | head -7 || exit 1
done; done
