#!/bin/bash
# Timing ablations (ablation build) for the tiles in TILES on the shapes in ONLY.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp LIB=0
export C2D_LIB="$GRAFT_REPO_ROOT/clap2diffusion_amd/libc2d_hip_abl.so"
for t in $TILES; do
  for a in ${ABLS:-0 1 2 3}; do
    echo "== tile $t abl $a"
    C2D_GEMM_TILE=$t C2D_GEMM_ABL=$a timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v amdgpu | cut -c1-60 || exit 1
  done
done
