#!/bin/bash
# Intra-workgroup split-K tiles 80 / 81: forced-tile parity, then graph-replayed (tile, split) sweeps of the
# level-2 / level-3 shapes at the three batches (c3 N = 16, c2 N = 2, c5 N = 8 at 96^2).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/kg
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "every_dma_tile_forced and (80 or 81)" > gpurun_out/kg/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/kg/pytest.log; [ $rc -eq 0 ] || exit $rc
T=${TILES:-80,81,8,9,7,3,41}
S=${SPLITS:-1,2,3,4,6,8,12}
for args in "--batch 8" "--batch 1" "--batch 4 --res 96"; do
  for lv in L2 L3 L1; do
    timeout -k 10 400 python -u scripts/sweep_tiles_graph.py $args --only "$lv " --tiles $T --splits $S \
      >> gpurun_out/kg/sweep_$(echo $args | tr -d ' -').txt 2>&1 || exit 1
  done
  grep -v amdgpu.ids gpurun_out/kg/sweep_$(echo $args | tr -d ' -').txt
done
