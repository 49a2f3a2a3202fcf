#!/bin/bash
# Round profile set: --kernel-trace --stats of the dominant conv and the d=40 attention
# alone (scripts/roof_kernel.py / roof_attn.py), then the PMC counter groups of
# scripts/gpu_counters.sh for both.  Output: gpurun_out/pmc/ (counters) and
# gpurun_out/roof/ (stats CSVs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/roof
for w in kernel attn; do
  rm -rf /tmp/roof_$w
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/roof_$w -o r -- python3 -u scripts/roof_$w.py 20 > gpurun_out/roof/$w.log 2>&1 || { echo "roof $w failed"; tail -5 gpurun_out/roof/$w.log; exit 1; }
  cp $(find /tmp/roof_$w -name "*kernel_stats.csv" | head -1) gpurun_out/roof/${w}_kernel_stats.csv
  tail -2 gpurun_out/roof/$w.log
done
NAMES="conv attn" bash scripts/gpu_counters.sh
