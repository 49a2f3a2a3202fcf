#!/bin/bash
# GPU tests (PYTEST_K subset or all), the per-shape GEMM breakdown, then the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
K=()
[ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread "${K[@]}" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/unet_shapes.py > gpurun_out/shapes.log 2>&1 || { echo "shapes rc $?"; tail -20 gpurun_out/shapes.log; exit 1; }
grep -v "^\[W\|^W20\|amdgpu.ids" gpurun_out/shapes.log | head -${SHAPES_LINES:-30}
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
