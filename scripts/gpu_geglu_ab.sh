#!/bin/bash
# GEGLU epilogue A/B: packed-pair math (libc2d_hip.so) vs per-element (libc2d_hip_gscalar.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "geglu" 2>&1 | tail -1 || exit 1
for rep in 1 2 3; do
  for v in pk gscalar; do
    lib=clap2diffusion_amd/libc2d_hip.so; [ $v = gscalar ] && lib=clap2diffusion_amd/libc2d_hip_gscalar.so
    for shp in "1 64 320 2560" "1 32 640 5120" "1 16 1280 10240"; do
      C2D_LIB=$PWD/$lib TAG=$v timeout -k 10 60 python -u scripts/time_gemm.py $shp --geglu || exit 1
    done
  done
done
