#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of one c3 batch and one c2 image.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c3 -o c3 -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/prof/c3_stdout.log 2> gpurun_out/prof/c3_stderr.log || { echo "c3 prof rc $?"; tail -5 gpurun_out/prof/c3_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c3 -name "*kernel_trace.csv" | head -1) 2 > gpurun_out/prof/c3_by_kernel.txt
cp $(find $P/c3 -name "*kernel_stats.csv" | head -1) gpurun_out/prof/c3_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/prof/c2_stdout.log 2> gpurun_out/prof/c2_stderr.log || { echo "c2 prof rc $?"; tail -5 gpurun_out/prof/c2_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c2 -name "*kernel_trace.csv" | head -1) 2 > gpurun_out/prof/c2_by_kernel.txt
head -16 gpurun_out/prof/c3_by_kernel.txt; head -14 gpurun_out/prof/c2_by_kernel.txt
