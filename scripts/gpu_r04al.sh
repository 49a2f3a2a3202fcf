#!/bin/bash
# Round 4, final .so: smoke(), the conv / GroupNorm / audio kernel tests, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04al; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; cut -c1-300 $O/bench.json; exit $rc
