#!/bin/bash
# c2: GroupNorm apply workgroups per launch below 8 images (the moments / fold apply): 512 / 1024 (main) / 2048,
# graph-replayed GroupNorm shapes at N = 2 and the bench's c2 latency, alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
VARIANTS="ap512:C2D_LIB=clap2diffusion_amd/libc2d_hip_ap512.so main:C2D_LIB=clap2diffusion_amd/libc2d_hip.so ap2048:C2D_LIB=clap2diffusion_amd/libc2d_hip_ap2048.so" \
  ROUNDS=2 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
