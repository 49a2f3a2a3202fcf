#!/bin/bash
# Ping-pong / 32x32 kernel timing ablations on the UNet GEMM shapes (ablation library:
# python -m clap2diffusion_amd.build --ablation on the CPU side): C2D_GEMM_ABL 0 = full,
# 4 = no epilogue, 1 = no DMA issue, 2 = no MFMA (results invalid for 1 / 2 / 4).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export C2D_LIB="$GRAFT_REPO_ROOT/clap2diffusion_amd/libc2d_hip_abl.so"
test -f "$C2D_LIB" || { echo "missing $C2D_LIB"; exit 1; }
for a in ${ABLS:-0 4 1 2}; do
  echo "== C2D_GEMM_ABL=$a"
  C2D_GEMM_ABL=$a timeout -k 10 200 python -u scripts/ab_tiles.py --shapes "${SHAPES:-geglu0,qkv0,conv0}" \
    --plans "${PLANS:-0,41:1}" --rounds 3 2>&1 | grep -v "amdgpu.ids" || exit 1
done
