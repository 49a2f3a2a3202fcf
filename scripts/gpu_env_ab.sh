#!/bin/bash
# Env-switch A/Bs on one box: GroupNorm apply workgroup count (graph-replayed GN shapes), then the
# bench line with and without C2D_GEMM_LDSEPI=0 (GEGLU direct epilogue), alternated three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for b in 2048 1024 4096; do
  echo "== C2D_GN_APPLY_BLOCKS=$b"
  C2D_GN_APPLY_BLOCKS=$b timeout -k 10 120 python -u scripts/bench_norm_graph.py 2>&1 | grep "^GN" | head -4 || exit 1
done
for r in 1 2 3; do
  for E in 1 0; do
    echo "== C2D_GEMM_LDSEPI=$E (round $r)"
    C2D_GEMM_LDSEPI=$E timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-configs 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('img/s', d['value'])" || exit 1
  done
done
