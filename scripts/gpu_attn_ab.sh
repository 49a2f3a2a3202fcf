#!/bin/bash
# Attention parity tests, then the attention microbench with each softmax variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k attention -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_attn.log | tail -20
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  echo "C2D_ATTN_NEGC=$v"
  C2D_ATTN_NEGC=$v timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
done
