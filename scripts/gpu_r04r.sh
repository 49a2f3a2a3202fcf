#!/bin/bash
# Round 4: raw kernel trace of one c2 generation (B = 1) for neighbour analysis of the small
# copyBuffer launches (which graph they sit in).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > $O/c2_stdout.log 2> $O/c2_stderr.log || { echo "c2 prof rc $?"; tail -5 $O/c2_stderr.log; exit 1; }
gzip -c $(find $P/c2 -name "*kernel_trace.csv" | head -1) > $O/c2_kernel_trace.csv.gz
ls -la $O
