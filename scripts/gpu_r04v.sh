#!/bin/bash
# Round 4: ping-pong residual / temb epilogue, compact (default) vs prefetch form (libc2d_hip_epf.so):
# kernel tests on the variant, then per-shape timings, two alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04v; mkdir -p $O
C2D_LIB=$PWD/clap2diffusion_amd/libc2d_hip_epf.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "epilogue_operand or padded_source or every_dma_tile_forced or split_k" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for L in libc2d_hip libc2d_hip_epf; do
    echo "== lib $L round $r"
    C2D_LIB=$PWD/clap2diffusion_amd/$L.so timeout -k 10 200 python -u scripts/ab_tiles.py --shapes conv0p,convt0p,upconv0p,proj0,conv1,conv2,qkv0 --plans 0 --rounds 3 2>/dev/null | grep -v amdgpu || exit 1
  done
done
