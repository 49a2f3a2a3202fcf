#!/bin/bash
# Round 4: the row-ring 3x3 conv (tile 42) and the zero-bordered GroupNorm: new kernel tests,
# the c3-batch UNet vs oracle, then timings against the stock tile 40, then the ablations of r04b.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
true || timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "padded_source or groupnorm_pad or cancelling or fully_masked or every_dma_tile_forced" > $O/pytest_k.log 2>&1
rc=$?; echo "pytest kernels exit $rc"; tail -3 $O/pytest_k.log; grep -E "FAIL|Error" $O/pytest_k.log | head -20
[ $rc -eq 0 ] || exit $rc
true || timeout -k 10 400 python -u -m pytest tests/test_unet_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "c3_batch or step_matches_oracle" > $O/pytest_u.log 2>&1
rc=$?; echo "pytest unet exit $rc"; tail -3 $O/pytest_u.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ab_tiles.py --shapes conv0p,convt0p,upconv0p,conv0,upconv0 --plans 0,40:1 --rounds 5 \
  > $O/ab_conv.txt 2>&1 || { echo "ab rc $?"; tail -5 $O/ab_conv.txt; exit 1; }
grep -v amdgpu.ids $O/ab_conv.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err
rc=$?; tail -2 $O/bench.err; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04b.sh
