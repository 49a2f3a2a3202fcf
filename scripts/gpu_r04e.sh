#!/bin/bash
# Round 4: tile 42 with the shift-conflict-free A swizzle (rr_swz, 80-row slots) vs the previous
# build (standard swizzle, 2-way conflicts at kx = 1, 2), same box, two alternations; parity first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
L=$PWD/clap2diffusion_amd
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "padded_source or groupnorm_pad" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in _old42 ""; do
    echo "== lib libc2d_hip$v.so round $r"
    C2D_LIB=$L/libc2d_hip$v.so timeout -k 10 120 python -u scripts/ab_tiles.py --shapes conv0p,convt0p,upconv0p,conv0 --plans 0 --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
  done
done > $O/ab.txt
cat $O/ab.txt
