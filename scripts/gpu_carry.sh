#!/bin/bash
# K = 320 GEGLU panel GEMM with each column block's epilogue carried into the next block's K loop
# (C2D_TUNE_PANEL_CARRY=1, variant build libc2d_hip_carry.so): the panel / GEGLU / UNet / bench-workload
# tests on the variant, then graph-replayed GEMM shapes and the bench line, same box, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
[ -n "$NOTEST" ] || VARIANTS="carry:C2D_LIB=clap2diffusion_amd/libc2d_hip_carry.so" \
  PYTEST_K="panel_gemm or geglu or unet_step_c3 or unet_step_c5 or bench_c3" ROUNDS=0 bash scripts/gpu_ab.sh || exit 1
VARIANTS="main:C2D_LIB=clap2diffusion_amd/libc2d_hip.so carry:C2D_LIB=clap2diffusion_amd/libc2d_hip_carry.so" \
  CMD=shapes SHAPES_LINES=14 ROUNDS=1 bash scripts/gpu_ab.sh || exit 1
VARIANTS="main:C2D_LIB=clap2diffusion_amd/libc2d_hip.so carry:C2D_LIB=clap2diffusion_amd/libc2d_hip_carry.so" \
  ROUNDS=2 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
