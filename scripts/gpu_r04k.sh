#!/bin/bash
# Round 4: carried-epilogue store placement A/B (C2D_PPS_DEFER / C2D_PPS_PH5 variant builds)
# on the tile-50 shapes, two alternations of the libraries on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
for r in 1 2; do
  for L in libc2d_hip libc2d_hip_d1p2 libc2d_hip_d1p4 libc2d_hip_d2p4 libc2d_hip_d0p4; do
    echo "== lib $L round $r" >> $O/ab.txt
    C2D_LIB=$PWD/clap2diffusion_amd/$L.so timeout -k 10 240 python -u scripts/ab_tiles.py \
      --shapes geglu0,geglu1,qkv0,toq0,qkv1,toq1 --plans 0,50:1 --rounds 3 >> $O/ab.txt 2>&1 || { tail -5 $O/ab.txt; exit 1; }
  done
done
grep -v amdgpu.ids $O/ab.txt > $O/ab_clean.txt
echo done
