#!/bin/bash
# Round 4: PMC passes (the round-3 GEMM-family set + the tile-42 dominant conv), then plan sweeps
# of the GEMM-family shapes over every eligible tile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
NAMES="geglu0 qkv0 res0 l2res conv0p conv0" bash scripts/gpu_gemm_counters.sh > $O/counters.log 2>&1 || { tail -20 $O/counters.log; exit 1; }
cp -r gpurun_out/gemmpmc $O/ 2>/dev/null
timeout -k 10 300 python -u scripts/ab_tiles.py --shapes geglu0,geglu1 --plans 0,25:1,41:1,1:1,28:1 --rounds 3 > $O/sweep_geglu.txt 2>&1 || { tail -3 $O/sweep_geglu.txt; exit 1; }
timeout -k 10 300 python -u scripts/ab_tiles.py --shapes qkv0,toq0,proj0 --plans 0,41:1,25:1,7:1,28:1,1:1 --rounds 3 > $O/sweep_l0.txt 2>&1 || { tail -3 $O/sweep_l0.txt; exit 1; }
timeout -k 10 300 python -u scripts/ab_tiles.py --shapes toq2,proj2 --plans 0,7:1,9:1,2:1,41:2,40:2,7:2,8:2 --rounds 3 > $O/sweep_l2.txt 2>&1 || { tail -3 $O/sweep_l2.txt; exit 1; }
grep -v amdgpu.ids $O/sweep_*.txt
