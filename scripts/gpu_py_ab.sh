#!/bin/bash
# Same-box A/B of two Python trees over one library: ab/ (an older checkout with its own bench.py and a
# copy of the .so) vs the repo root, bench line alternated three times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2 3; do
  for D in ab .; do
    echo "== $D (round $r)"
    timeout -k 10 300 python -u $D/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-configs 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('img/s', d['value'])" || exit 1
  done
done
