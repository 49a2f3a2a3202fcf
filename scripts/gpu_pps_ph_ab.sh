#!/bin/bash
# pps (tile 50) 4-phase vs 2-phase K steps: parity of the 2-phase build, then same-box timing A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
C2D_LIB=$PWD/clap2diffusion_amd/libc2d_hip_ph2.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "persistent or geglu" > gpurun_out/ph/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/ph/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base ph2; do
    lib=clap2diffusion_amd/libc2d_hip.so; [ $v = ph2 ] && lib=clap2diffusion_amd/libc2d_hip_ph2.so
    echo "== $v"
    C2D_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/sweep_tiles_graph.py --batch 8 --only "L0 geglu" --tiles 25 --splits 1 2>&1 | grep geglu || exit 1
  done
done
