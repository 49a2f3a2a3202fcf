#!/bin/bash
# CFG-prefix parity (half copies), attention young-half priority A/B (variant library), c3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_unet_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cfg_shared or c3_batch or graph or 10_steps" > gpurun_out/ab/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/ab/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base yprio; do
    lib=clap2diffusion_amd/libc2d_hip.so; [ $v = yprio ] && lib=clap2diffusion_amd/libc2d_hip_yprio.so
    C2D_LIB=$PWD/$lib TAG=$v timeout -k 10 120 python -u scripts/attn_d40_check.py 2>&1 | grep "^$v" || exit 1
  done
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > gpurun_out/ab/bench.json 2> gpurun_out/ab/bench.err
rc=$?; tail -2 gpurun_out/ab/bench.err; cat gpurun_out/ab/bench.json; exit $rc
