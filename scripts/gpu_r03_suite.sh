#!/bin/bash
# Full -m gpu suite (parity figures -> gpurun_out/parity_metrics.tsv), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 850 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc
