#!/bin/bash
# Same-box A/B of two library builds (C2D_LIB): GEMM kernel tests on B, the per-shape UNet GEMM
# breakdown for each, then the bench line for each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
A=${A:-clap2diffusion_amd/libc2d_ab_old.so}; B=${B:-clap2diffusion_amd/libc2d_hip.so}
if [ -z "$NOTEST" ]; then
  C2D_LIB=$PWD/$B timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_k.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
fi
for L in $A $B; do
  echo "== shapes $L"
  C2D_LIB=$PWD/$L timeout -k 10 300 python -u scripts/unet_shapes.py > gpurun_out/shapes_$(basename $L).log 2>&1 || { echo "shapes rc $?"; exit 1; }
  grep -v "^\[W\|^W20\|amdgpu.ids" gpurun_out/shapes_$(basename $L).log | head -${SHAPES_LINES:-24}
done
for r in 1 2; do
  for L in $A $B; do
    echo "== bench $L (round $r)"
    C2D_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-configs 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('img/s', d['value'], 'dom us', d['roofline']['avg_us'])" || exit 1
  done
done
