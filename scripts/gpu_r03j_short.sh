#!/bin/bash
# Short final check of the third session's tree: the pipeline / golden / UNet GPU tests (the parts not
# yet run with the FF-out fold and fp16 split-K slabs together), smoke, then the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_golden_gpu.py tests/test_unet_gpu.py -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_short.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_short.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err
rc=$?; tail -3 gpurun_out/bench_j.err; cat gpurun_out/bench_j.json; exit $rc
