#!/bin/bash
# Bench A/B: commit 76d4add (ab/prev), this tree, this tree without the CFG-shared prefix at one latent per call
# (c2), this tree with the plain upsample; then the c2 trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PYTEST_K="upsample or unet_step_c3 or cfg_shared" NOAB=1 bash scripts/gpu_gnm.sh || exit $?
VARIANTS=${VARIANTS:-"prev:PYROOT=ab/prev new:C2D_CFG_PREFIX_MIN=1 nopre:C2D_CFG_PREFIX_MIN=2 noup:C2D_UP_PAD=0"} ROUNDS=2 \
  BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh || exit $?
NOBENCH=1 TRACES="c2" bash scripts/gpu_bench_prof.sh
