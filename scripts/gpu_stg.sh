#!/bin/bash
# Panel GEMM start stagger of waves 4-7 (C2D_TUNE_PANEL_STAGGER x 2048 cycles) re-measured with the carried GEGLU
# epilogue and waves 4-7 at s_setprio 1: 0 / 2 (main) / 4, GEMM shapes once, then the bench line, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
L=clap2diffusion_amd
V="stg0:C2D_LIB=$L/libc2d_hip_stg0.so main:C2D_LIB=$L/libc2d_hip.so stg4:C2D_LIB=$L/libc2d_hip_stg4.so"
VARIANTS="$V" CMD=shapes SHAPES_LINES=8 ROUNDS=1 bash scripts/gpu_ab.sh || exit 1
VARIANTS="$V" ROUNDS=2 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
