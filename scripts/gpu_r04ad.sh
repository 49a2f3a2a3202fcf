#!/bin/bash
# Round 4 evidence after the two-launch GroupNorm: the default bench line (PMC traffic + c1 CPU leg), then kernel traces of
# one c3 batch (B = 8) and one c2 image (B = 1), summarised per kernel family.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ad; mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c3 -o c3 -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > $O/c3_stdout.log 2> $O/c3_stderr.log || { echo "c3 prof rc $?"; tail -5 $O/c3_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c3 -name "*kernel_trace.csv" | head -1) 2 > $O/c3_by_kernel.txt
cp $(find $P/c3 -name "*kernel_stats.csv" | head -1) $O/c3_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > $O/c2_stdout.log 2> $O/c2_stderr.log || { echo "c2 prof rc $?"; tail -5 $O/c2_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c2 -name "*kernel_trace.csv" | head -1) 2 > $O/c2_by_kernel.txt
head -12 $O/c3_by_kernel.txt; head -12 $O/c2_by_kernel.txt
