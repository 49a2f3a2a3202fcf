#!/bin/bash
# Static s_setprio 1 for waves 4-7: 8-wave d = 40 attention blocks (aprio), the panel GEMM (pprio), and the
# panel GEMM with its GEGLU epilogue carried (cp = carry + pprio): attention shapes, then the bench line,
# same box, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
L=clap2diffusion_amd
VARIANTS="main:C2D_LIB=$L/libc2d_hip.so aprio:C2D_LIB=$L/libc2d_hip_aprio.so" CMD=attn ROUNDS=2 bash scripts/gpu_ab.sh || exit 1
VARIANTS="main:C2D_LIB=$L/libc2d_hip.so aprio:C2D_LIB=$L/libc2d_hip_aprio.so pprio:C2D_LIB=$L/libc2d_hip_pprio.so cp:C2D_LIB=$L/libc2d_hip_cp.so" \
  ROUNDS=2 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
