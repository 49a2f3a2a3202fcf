#!/bin/bash
# Graph-timed (tile, split) sweep at the c3 (N = 16), c2 (N = 2) and c5 (N = 8, 96^2) batches.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
run() {  # tag, args
  timeout -k 10 400 python -u scripts/sweep_tiles_graph.py $2 $SWEEP_ARGS > gpurun_out/sweep/$1.log 2>&1 || { echo "$1 rc $?"; tail -20 gpurun_out/sweep/$1.log; exit 1; }
  grep -v "^\[W\|^W20\|amdgpu.ids" gpurun_out/sweep/$1.log
}
run b1 "--batch 1" && run b4r96 "--batch 4 --res 96" && run b8 "--batch 8"
