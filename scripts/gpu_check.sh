#!/bin/bash
# GPU tests + norm microbench (rocprof stats) + bench. Stops at the first fault / timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$MICRO" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pm -o m -- python3 -u $MICRO > gpurun_out/micro.log 2>&1 || { echo "micro failed"; tail gpurun_out/micro.log; exit 1; }
  cp /tmp/pm/m_kernel_stats.csv gpurun_out/micro_stats.csv
  grep -v "^[WE]2026" gpurun_out/micro.log
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/micro_stats.csv')):
    print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5}  {r['Name'][:110]}\")
"
fi
timeout -k 10 400 python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
