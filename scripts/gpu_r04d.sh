#!/bin/bash
# Round 4: tile 42 phase count A/B (4 phases vs 2 phases with every DMA piece in phase 0), same box,
# two alternations; tile 40 on the unpadded source as the control.  Then tile-42 parity with PH = 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
L=$PWD/clap2diffusion_amd
for r in 1 2; do
  for v in "" _ph2; do
    echo "== lib libc2d_hip$v.so round $r"
    C2D_LIB=$L/libc2d_hip$v.so timeout -k 10 120 python -u scripts/ab_tiles.py --shapes conv0p,convt0p,upconv0p,conv0 --plans 0 --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab_ph.txt
cat $O/ab_ph.txt
C2D_LIB=$L/libc2d_hip_ph2.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "padded_source" > $O/pytest_ph2.log 2>&1; rc=$?; tail -2 $O/pytest_ph2.log; exit $rc
