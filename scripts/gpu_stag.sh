#!/bin/bash
# d = 40 attention with staggered halves: attention -m gpu tests, per-shape A/B against the lockstep build
# (libc2d_hip_stag0.so, -DC2D_TUNE_ATTN_STAG=0), then the bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PYTEST_K="attention or attn or gn_moments or unet_step or bench_c3" NOAB=1 bash scripts/gpu_gnm.sh || exit $?
V="lock:C2D_LIB=clap2diffusion_amd/libc2d_hip_stag0.so stag:C2D_LIB=clap2diffusion_amd/libc2d_hip.so"
VARIANTS="$V" ROUNDS=2 CMD=attn bash scripts/gpu_ab.sh || exit $?
VARIANTS="$V" ROUNDS=2 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
NOBENCH=1 TRACES="c2" bash scripts/gpu_bench_prof.sh
