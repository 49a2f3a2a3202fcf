#!/bin/bash
# Round 4, final tree: smoke(), then the default bench line (PMC traffic + c1 CPU leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; cat $O/bench.json; exit $rc
