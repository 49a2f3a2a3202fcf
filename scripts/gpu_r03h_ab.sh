#!/bin/bash
# Two A/B switches (read once per process): C2D_GN_WIDE_N (1024-thread single-launch GroupNorm for
# N <= 2 images) and C2D_SPLITK_F16 (split-K partials in fp16).  Parity tests with both on, the
# affected kernels off vs on, then the bench (c3 / c2 / c1 / c5) over the four combinations, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
C2D_GN_WIDE_N=2 C2D_SPLITK_F16=1 timeout -k 10 450 python -u -m pytest tests/test_kernels_gpu.py tests/test_unet_gpu.py \
  -x -v --timeout 300 --timeout-method thread -k "groupnorm or split or forced or matches_oracle or conv3x3" \
  > gpurun_out/h_tests.log 2>&1 || { tail -30 gpurun_out/h_tests.log; exit 1; }
tail -2 gpurun_out/h_tests.log
for n in 1 2; do
  for w in 0 2; do
    echo "== GN N=$n wide_n=$w"
    GN_N=$n C2D_GN_WIDE_N=$w timeout -k 10 120 python -u scripts/bench_norm_graph.py || exit 1
  done
done
for b in 8 1; do
  for f in 0 1; do
    echo "== C2D_SPLITK_F16=$f batch $b (the 'default' column is the planned split)"
    C2D_SPLITK_F16=$f timeout -k 10 200 python -u scripts/sweep_tiles_graph.py --batch $b --only 3x3 --tiles 40 --splits 1 || exit 1
  done
done
for r in 1 2; do
  for wf in "0 0" "2 0" "0 1" "2 1"; do
    set -- $wf
    C2D_GN_WIDE_N=$1 C2D_SPLITK_F16=$2 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc \
      > gpurun_out/h_$1$2.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/h_$1$2.json')); print('wide_n=$1 splitk_f16=$2 c3 %.4f img/s  c2 %.4f s  c1 %.4f s  c5 %.4f img/s' % (d['value'], d['c2_latency_s'], d['c1_gpu_latency_s'], d['c5_images_per_s']))"
  done
done
