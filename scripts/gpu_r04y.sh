#!/bin/bash
# Round 4: single-launch GroupNorm (gn_grid_kernel) -- GroupNorm tests, per-call graph timing
# against the multi-launch paths (C2D_GN_GRID 0 / 1 / 2) at N = 16 and N = 2, then the bench legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r04y
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "groupnorm or gn_silu" 2>&1 | grep -v amdgpu > gpurun_out/r04y/pytest_gn.txt
rc=$?; tail -3 gpurun_out/r04y/pytest_gn.txt; [ $rc -eq 0 ] || exit $rc
for n in 16 2; do for m in 0 1 2; do
  echo "== N=$n C2D_GN_GRID=$m"
  GN_N=$n C2D_GN_GRID=$m timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep -v amdgpu || exit 1
done; done
for m in 1 0; do
  echo "== bench C2D_GN_GRID=$m"
  C2D_GN_GRID=$m timeout -k 10 400 python -u bench.py 2>&1 | grep -v amdgpu | tail -1 | cut -c1-420 || exit 1
done
