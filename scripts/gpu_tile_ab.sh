#!/bin/bash
# Forced-tile parity tests, then the GEMM microbench for the default planner and for each
# tile id in TILES (C2D_GEMM_TILE), on the shapes in ONLY.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-every_dma_tile}" > gpurun_out/tile_tests.log 2>&1
rc=$?; tail -3 gpurun_out/tile_tests.log; [ $rc -eq 0 ] || exit $rc
export LIB=0
echo "== default"; timeout -k 10 200 python -u scripts/bench_gemm.py 2>&1 | grep -v amdgpu || exit 1
for t in $TILES; do
  echo "== tile $t"; C2D_GEMM_TILE=$t timeout -k 10 200 python -u scripts/bench_gemm.py 2>&1 | grep -v amdgpu || exit 1
done
