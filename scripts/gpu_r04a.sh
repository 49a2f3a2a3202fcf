#!/bin/bash
# Round 4, first GPU call: the changed / new kernel tests and the UNet-vs-oracle tests (tighter
# bars, fp32 split-K slabs), per-shape timings of the GEMM family, the bench line and a kernel
# trace of one c3 batch (the final tree's family split).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 $O/pytest.log; cp gpurun_out/parity_metrics.tsv $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/ab_tiles.py --shapes geglu0,geglu1,qkv0,qkv1,proj0,toq2,proj2,conv0,conv1,conv2 \
  --plans 0 --rounds 5 > $O/shapes.txt 2>&1 || { echo "shapes rc $?"; tail -5 $O/shapes.txt; exit 1; }
cat $O/shapes.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c3 -o c3 -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > $O/c3_stdout.log 2> $O/c3_stderr.log || { echo "c3 prof rc $?"; tail -5 $O/c3_stderr.log; exit 1; }
python3 scripts/kt_summary.py $(find $P/c3 -name "*kernel_trace.csv" | head -1) 2 > $O/c3_by_kernel.txt
cp $(find $P/c3 -name "*kernel_stats.csv" | head -1) $O/c3_kernel_stats.csv
head -40 $O/c3_by_kernel.txt
