#!/bin/bash
# Per-shape GEMM breakdown of one UNet call + forced-tile A/B of chosen shapes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/unet_shapes.py > gpurun_out/shapes.log 2>&1 || { echo "shapes rc $?"; tail -20 gpurun_out/shapes.log; exit 1; }
grep -v "^\[W\|^W20" gpurun_out/shapes.log | head -70
for t in ${TILES:-41 25}; do
  echo "== C2D_GEMM_TILE=$t ONLY=$ONLY"
  C2D_GEMM_TILE=$t LIB=0 ONLY="$ONLY" timeout -k 10 200 python -u scripts/bench_gemm.py 2>&1 | grep -v "^\[W\|^W20" || exit 1
done
