#!/bin/bash
# Timing ablation of forced implicit-GEMM plans (libc2d_hip_abl.so, C2D_GEMM_ABL bits; wrong
# results by design): 1 = no DMA after the prologue, 2 = no MFMA, 4 = no epilogue.
# SHAPES / PLANS / ABLS select the cases (scripts/ab_tiles.py names); build the ablation library
# first on the CPU side: python -m clap2diffusion_amd.build --ablation
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export C2D_LIB="$GRAFT_REPO_ROOT/clap2diffusion_amd/libc2d_hip_abl.so"
test -f "$C2D_LIB" || { echo "missing $C2D_LIB"; exit 1; }
for a in ${ABLS:-0 1 2 3 4}; do
  echo "== C2D_GEMM_ABL=$a"
  C2D_GEMM_ABL=$a timeout -k 10 120 python -u scripts/ab_tiles.py --shapes "${SHAPES:-conv0,qkv0}" \
      --plans "${PLANS:-40:0,60:0}" --rounds 3 2>&1 | grep -v amdgpu || exit 1
done
