#!/bin/bash
# Moments threaded through transformer outputs / downsamplers: tests, then a 3-arm same-box A/B and a c2 trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
NOAB=1 bash scripts/gpu_gnm.sh || exit $?
VARIANTS="base:PYROOT=ab/base prev:PYROOT=ab/prev new:C2D_GN_MOMENTS=1" ROUNDS=2 \
  BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh || exit $?
NOBENCH=1 TRACES="c2 c3" bash scripts/gpu_bench_prof.sh
