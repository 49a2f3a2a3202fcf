#!/bin/bash
# Round 4: fold-path apply workgroups 1024 (new default) vs 2048, bench legs alternated, then the GroupNorm tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do for ab in 1024 2048; do
  echo "== bench C2D_GN_FOLD_APPLY_BLOCKS=$ab round $r"
  C2D_GN_FOLD_APPLY_BLOCKS=$ab timeout -k 10 400 python -u bench.py --no-pmc --no-cpu-baseline 2>/dev/null | grep -v amdgpu | python3 scripts/bench_legs.py || exit 1
done; done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "groupnorm or gn_silu" 2>&1 | tail -1
