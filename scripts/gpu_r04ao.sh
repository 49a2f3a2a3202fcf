#!/bin/bash
# Round 4, final .so: the whole GPU suite, smoke(), the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ao; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; tail -2 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; cat $O/bench.json; exit $rc
