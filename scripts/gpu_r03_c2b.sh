#!/bin/bash
# c2-path parity (B = 1 / N = 2 UNet and pipeline tests), bench (c3 + side configs), c2 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or every_dma or groupnorm or gn_silu or dual_source" > gpurun_out/c2/pytest_k.log 2>&1 || { tail -5 gpurun_out/c2/pytest_k.log; exit 1; }; tail -1 gpurun_out/c2/pytest_k.log
timeout -k 10 400 python -u -m pytest tests/test_unet_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "batch1 or 10_steps or 16-981 or 32-501 or cfg_shared or c1_workload" > gpurun_out/c2/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/c2/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/c2/bench.json 2> gpurun_out/c2/bench.err
rc=$?; tail -2 gpurun_out/c2/bench.err; cat gpurun_out/c2/bench.json; [ $rc -eq 0 ] || exit $rc
P=/tmp/prof; rm -rf $P; mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/c2 -o c2 -- python3 -u bench.py --batch 1 --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > gpurun_out/c2/prof_stdout.log 2> gpurun_out/c2/prof_stderr.log || { echo "c2 prof rc $?"; exit 1; }
python3 scripts/kt_summary.py $(find $P/c2 -name "*kernel_trace.csv" | head -1) 2 > gpurun_out/c2/c2_by_kernel.txt
head -40 gpurun_out/c2/c2_by_kernel.txt
