#!/bin/bash
# Tests of the moments fold / combine and the buffer-load attention staging, then the attention shapes A/B
# against the -DC2D_TUNE_ATTN_BUFLD=0 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PYTEST_K="gn_moments or groupnorm or attention or attn or unet_step or cfg_shared or bench_c3" NOAB=1 bash scripts/gpu_gnm.sh || exit $?
VARIANTS="buf0:C2D_LIB=clap2diffusion_amd/libc2d_hip_buf0.so main:C2D_LIB=clap2diffusion_amd/libc2d_hip.so" ROUNDS=2 CMD=attn \
  bash scripts/gpu_ab.sh
