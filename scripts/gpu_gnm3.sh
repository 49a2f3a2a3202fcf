#!/bin/bash
# Moments fold without per-block divisions + 16-row combine blocks: tests, 3-arm A/B (76d4add tree, this tree,
# this tree without the CFG-shared prefix at one latent), c2 trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PYTEST_K="gn_moments or groupnorm or unet_step or cfg_shared or bench_c3 or pipeline_matches" NOAB=1 bash scripts/gpu_gnm.sh || exit $?
VARIANTS="prev:PYROOT=ab/prev new:C2D_CFG_PREFIX_MIN=1 nopre:C2D_CFG_PREFIX_MIN=2" ROUNDS=2 \
  BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh || exit $?
NOBENCH=1 TRACES="c2" bash scripts/gpu_bench_prof.sh
