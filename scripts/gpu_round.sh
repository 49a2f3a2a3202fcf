#!/bin/bash
# One GPU call: gpu tests, then the default bench.  Stops at a fault / abort / timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
