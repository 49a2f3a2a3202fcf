#!/bin/bash
# GEGLU panel epilogue on packed pairs: GEGLU tests, then the GEGLU shapes (graph-replayed, planner's plan) and the
# bench against the -DC2D_TUNE_PANEL_PK=0 build, alternated twice on one box; ln0 = the K = 640 LayerNorm fold off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PYTEST_K="geglu or panel or layernorm_fold or unet_step_c3 or bench_c3" NOAB=1 bash scripts/gpu_gnm.sh || exit $?
for r in 1 2; do
  for arm in pk0:clap2diffusion_amd/libc2d_hip_pk0.so pk1:clap2diffusion_amd/libc2d_hip.so; do
    echo "== ${arm%%:*} (round $r)"
    for b in "--batch 8" "--batch 1" "--batch 4 --res 96"; do
      C2D_LIB=$PWD/${arm#*:} timeout -k 10 200 python -u scripts/sweep_tiles_graph.py $b --only geglu --tiles 70 --splits 1 \
        2>&1 | grep -v amdgpu.ids || exit 1
    done
  done
done
VARIANTS="pk0:C2D_LIB=clap2diffusion_amd/libc2d_hip_pk0.so pk1:C2D_LIB=clap2diffusion_amd/libc2d_hip.so ln0:C2D_LN_FOLD640=0" ROUNDS=2 \
  BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-pmc" bash scripts/gpu_ab.sh
