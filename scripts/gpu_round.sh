#!/bin/bash
# One GPU call: gpu tests (PYTEST_K selects a subset), then the bench unless NOBENCH=1.
# Stops at a fault / abort / timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
K=()
[ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${K[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -3; tail -5 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
[ -n "$NOBENCH" ] && exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-500} python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
