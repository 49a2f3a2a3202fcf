#!/bin/bash
# GEMM timing ablation (C2D_GEMM_ABL bits; results invalid, timing only):
# 1 = no DMA issue, 2 = no MFMA, 4 = no epilogue (m32), 8 = with 2: no fragment reads (m32).
# Needs the ablation build (python -m clap2diffusion_amd.build --ablation, on the CPU side):
# the production libc2d_hip.so compiles the switches out.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export C2D_LIB="$GRAFT_REPO_ROOT/clap2diffusion_amd/libc2d_hip_abl.so"
test -f "$C2D_LIB" || { echo "missing $C2D_LIB"; exit 1; }
for a in ${ABLS:-0 1 2 3}; do
  echo "== abl $a"
  C2D_GEMM_ABL=$a ONLY="${ONLY:-L0 conv3x3 320,L1 conv3x3 640,L0 proj,L1 qkv,L0 geglu}" timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v amdgpu || exit 1
done
