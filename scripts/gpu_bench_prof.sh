#!/bin/bash
# Default bench line (BENCH_ARGS), then a rocprofv3 kernel trace of one short bench step,
# summarised per kernel+grid into gpurun_out/prof/bench_by_kernel.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
if [ -z "$NOBENCH" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-500} python -u bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; tail -4 gpurun_out/bench.err; cat gpurun_out/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
[ -n "$NOPROF" ] && exit 0
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/bench -o bench -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/prof/bench_stdout.log 2> gpurun_out/prof/bench_stderr.log || { echo "bench prof rc $?"; tail -20 gpurun_out/prof/bench_stderr.log; exit 1; }
for f in $(find $P -name "*stats.csv"); do cp $f gpurun_out/prof/; done
python3 scripts/kt_summary.py $(find $P -name "*kernel_trace.csv" | head -1) 2 > gpurun_out/prof/bench_by_kernel.txt
gzip -c $(find $P -name "*kernel_trace.csv" | head -1) > gpurun_out/prof/bench_kernel_trace.csv.gz
head -45 gpurun_out/prof/bench_by_kernel.txt
