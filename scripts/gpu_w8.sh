#!/bin/bash
# d = 40 attention: 4-wave blocks when the 8-wave grid would be under two blocks per CU (c2): attention tests, the
# attention shapes and the bench against the always-8-wave build (-DC2D_TUNE_ATTN_W8_MIN=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
true
V="w8all:C2D_LIB=clap2diffusion_amd/libc2d_hip_w8all.so main:C2D_LIB=clap2diffusion_amd/libc2d_hip.so"
VARIANTS="$V" ROUNDS=2 CMD=attn bash scripts/gpu_ab.sh || exit $?
VARIANTS="$V" ROUNDS=2 BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
