#!/bin/bash
# Round 4: where the GEMM-family time goes.  (1) timing ablations (libc2d_hip_abl.so:
# C2D_GEMM_ABL 1 = no DMA after the prologue, 2 = no MFMA, 4 = no epilogue / carried epilogue,
# 8 = pps: epilogue math without stores) on the dominant conv and the L0 1x1 / GEGLU shapes;
# (2) the persistent carried-epilogue tile 50 on the plain-output projections.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
for abl in 0 1 2 4 8 3; do
  echo "== C2D_GEMM_ABL=$abl"
  C2D_LIB=$PWD/clap2diffusion_amd/libc2d_hip_abl.so C2D_GEMM_ABL=$abl timeout -k 10 120 python -u scripts/ab_tiles.py \
    --shapes conv0,conv0p,qkv0,proj0,geglu0,toq2 --plans 0 --rounds 3 || exit 1
done > $O/abl.txt 2>&1
cat $O/abl.txt | grep -v amdgpu.ids
timeout -k 10 200 python -u scripts/ab_tiles.py --shapes qkv0,toq0,qkv1,toq1,qkv2,toq2 --plans 0,50:0 --rounds 5 \
  > $O/pps_plain.txt 2>&1 || exit 1
cat $O/pps_plain.txt | grep -v amdgpu.ids
