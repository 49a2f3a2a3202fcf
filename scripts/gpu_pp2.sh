#!/bin/bash
# d = 40 ping-pong attention: correctness + timing per C2D_ATTN_PP2 setting, alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pp2
for rep in 1 2; do
  for pp in 0 2 4; do
    C2D_ATTN_PP2=$pp timeout -k 10 120 python -u scripts/attn_pp2_check.py > gpurun_out/pp2/pp$pp.$rep.log 2>&1 || { echo "pp$pp rc $?"; tail -20 gpurun_out/pp2/pp$pp.$rep.log; exit 1; }
    grep PP2 gpurun_out/pp2/pp$pp.$rep.log
  done
done
