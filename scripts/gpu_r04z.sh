#!/bin/bash
# Round 4: two-launch GroupNorm (group-pair partials + apply that folds them; no finalize launch) --
# bench legs A/B against the three-launch path (C2D_GN_FOLD 1 / 0), alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do for m in 1 0; do
  echo "== bench C2D_GN_FOLD=$m round $r"
  C2D_GN_FOLD=$m timeout -k 10 400 python -u bench.py --no-pmc --no-cpu-baseline 2>/dev/null | grep -v amdgpu | python3 scripts/bench_legs.py || exit 1
done; done
