#!/bin/bash
# Producer-emitted GroupNorm moments: the -m gpu subset that covers them (kernel forms, the UNet and the bench
# workload against the oracle), then a same-box A/B of the round's start (ab/base) against the tree with and
# without the moments path (C2D_GN_MOMENTS).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "${PYTEST_K:-gn_moments or dma_tile_forced or unet_step or cfg_shared or bench_c3 or groupnorm}" \
  > gpurun_out/pytest_gnm.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gnm.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_gnm.log | head -30; exit $rc; }
[ -n "$NOAB" ] && exit 0
VARIANTS=${VARIANTS:-"base:PYROOT=ab/base new:C2D_GN_MOMENTS=1 nogn:C2D_GN_MOMENTS=0"} ROUNDS=${ROUNDS:-2} \
  BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
