#!/bin/bash
# pp16 (tiles 40 / 41) 4-phase vs 2-phase K steps: parity of the 2-phase build, then same-box timing A/B
# over the c3 shapes (default plans), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
C2D_LIB=$PWD/clap2diffusion_amd/libc2d_hip_pp2.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "tile or conv3x3 or epilogue or dual or linear or geglu or persistent" > gpurun_out/ph/pytest_pp2.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/ph/pytest_pp2.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base pp2; do
    lib=clap2diffusion_amd/libc2d_hip.so; [ $v = pp2 ] && lib=clap2diffusion_amd/libc2d_hip_pp2.so
    echo "== $v"
    C2D_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/sweep_tiles_graph.py --batch 8 --tiles 40 --splits 1 2>&1 | grep " us " | cut -c1-60 || exit 1
  done
done
