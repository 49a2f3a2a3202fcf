#!/bin/bash
# Per-shape GEMM timings for each forced tile config (C2D_GEMM_TILE), one process each.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
for t in ${TILES:-0 1 2 3 7}; do
  echo "== tile $t"
  C2D_GEMM_TILE=$t timeout -k 10 150 python scripts/bench_gemm.py || exit 1
done
