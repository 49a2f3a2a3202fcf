#!/bin/bash
# ff.net.2 folded into proj_out (C2D_FOLD_FF_OUT, read at import): the fold's parity tests, the
# folded GEMM shapes swept per batch, then c3 / c2 / c5 alternated with the fold off and on.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_unet_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "fold or matches_oracle" > gpurun_out/fold_tests.log 2>&1 || { tail -30 gpurun_out/fold_tests.log; exit 1; }
tail -3 gpurun_out/fold_tests.log
for b in 8 1; do
  timeout -k 10 300 python -u scripts/sweep_tiles_graph.py --batch $b --only fold --tiles 40,41,25,7,1,2,3,8,9 \
    --splits 1,2,3,4,6,8,12,16 || exit 1
done
timeout -k 10 300 python -u scripts/sweep_tiles_graph.py --batch 4 --res 96 --only fold --tiles 40,41,25,7,1,2,3,8,9 \
  --splits 1,2,3,4,6,8 || exit 1
for r in 1 2; do
  for f in 0 1; do
    C2D_FOLD_FF_OUT=$f timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc \
      > gpurun_out/fold_$f.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/fold_$f.json')); print('fold=$f c3 %.4f img/s  c2 %.4f s  c5 %.4f img/s' % (d['value'], d['c2_latency_s'], d['c5_images_per_s']))"
  done
done
