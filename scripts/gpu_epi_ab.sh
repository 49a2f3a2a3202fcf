#!/bin/bash
# 32x32-tile epilogue A/B: direct from the accumulators (C2D_GEMM_LDSEPI=0) vs LDS-staged (1).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in 0 1; do
  C2D_GEMM_LDSEPI=$e timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv or gemm or linear or geglu or m32" --timeout 120 --timeout-method thread > gpurun_out/epi_t$e.log 2>&1
  rc=$?; echo "tests LDSEPI=$e: $(tail -1 gpurun_out/epi_t$e.log)"; [ $rc -eq 0 ] || exit $rc
done
for e in 0 1; do
  echo "== C2D_GEMM_LDSEPI=$e"
  C2D_GEMM_LDSEPI=$e ONLY="${ONLY:-L0 conv3x3 320,L0 up conv,L0 geglu,L0 GEGLU act,L0 qkv,L0 proj,L0 ff2,L1 geglu,L1 GEGLU act}" timeout -k 10 120 python scripts/bench_gemm.py 2>&1 | grep -v amdgpu || exit 1
done
