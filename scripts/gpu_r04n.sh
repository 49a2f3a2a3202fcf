#!/bin/bash
# Round 4: GroupNorm-pad apply with unconditional loads (tests + c3 trace), and the device-copy census
# of one denoise step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "groupnorm or conv3x3_padded" -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/copy_census.py --batch 1 > $O/copy_census_b1.txt 2>&1 || { echo "census rc $?"; tail -20 $O/copy_census_b1.txt; exit 1; }
grep -v amdgpu.ids $O/copy_census_b1.txt | head -60
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c3 -o c3 -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > $O/c3_stdout.log 2> $O/c3_stderr.log || { echo "c3 prof rc $?"; tail -5 $O/c3_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c3 -name "*kernel_trace.csv" | head -1) 2 > $O/c3_by_kernel.txt
head -14 $O/c3_by_kernel.txt; grep gn_apply $O/c3_by_kernel.txt
