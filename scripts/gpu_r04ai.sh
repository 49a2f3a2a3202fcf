#!/bin/bash
# Round 4: image split of a quantisation tail (c5's level-0 convs), per-call timing A/B, then the c5 bench leg
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for m in 0 1; do C2D_TAIL_SPLIT=$m timeout -k 10 200 python -u scripts/tail_split_ab.py 2>&1 | grep -v amdgpu || exit 1; done
for r in 1 2; do for m in 1 0; do
  echo "== bench C2D_TAIL_SPLIT=$m round $r"
  C2D_TAIL_SPLIT=$m timeout -k 10 400 python -u bench.py --no-pmc --no-cpu-baseline 2>/dev/null | grep -v amdgpu | python3 scripts/bench_legs.py || exit 1
done; done
