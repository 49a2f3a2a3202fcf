#!/bin/bash
# Round bench line (default flags) + rocprofv3 kernel trace of a one-step bench + dominant-kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/roof
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc $?"; tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
NOBENCH=1 bash scripts/gpu_bench_prof.sh || exit 1
rm -rf /tmp/roof_kernel
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/roof_kernel -o r -- python3 -u scripts/roof_kernel.py 20 > gpurun_out/roof/kernel.log 2>&1 || { echo "roof failed"; exit 1; }
cp $(find /tmp/roof_kernel -name "*kernel_stats.csv" | head -1) gpurun_out/roof/kernel_kernel_stats.csv
tail -2 gpurun_out/roof/kernel.log
