#!/bin/bash
# Round-3 re-survey: per-shape GEMM breakdown of one UNet call at the c3 batch (N = 16) and
# the c2 batch (N = 2), then a kernel trace of the c2 configuration (B = 1, 512^2, 50 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/survey
timeout -k 10 240 python -u scripts/unet_shapes.py --batch 8 > gpurun_out/survey/shapes_b8.log 2>&1 || { echo "shapes b8 rc $?"; tail -20 gpurun_out/survey/shapes_b8.log; exit 1; }
timeout -k 10 240 python -u scripts/unet_shapes.py --batch 1 > gpurun_out/survey/shapes_b1.log 2>&1 || { echo "shapes b1 rc $?"; tail -20 gpurun_out/survey/shapes_b1.log; exit 1; }
P=/tmp/prof_c2; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/survey/c2_stdout.log 2> gpurun_out/survey/c2_stderr.log || { echo "c2 prof rc $?"; tail -20 gpurun_out/survey/c2_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P -name "*kernel_trace.csv" | head -1) 2 > gpurun_out/survey/c2_by_kernel.txt
grep -v "^\[W\|^W20" gpurun_out/survey/shapes_b8.log | head -40
grep -v "^\[W\|^W20" gpurun_out/survey/shapes_b1.log | head -40
head -30 gpurun_out/survey/c2_by_kernel.txt
