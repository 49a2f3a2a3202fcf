#!/bin/bash
# Round 4: two-workgroups-per-CU tiles (8 = 128x160, 9 = 64x160) against the planner's tiles on the
# epilogue-bound K = 320 GEMMs at c3 (N = 16, 64^2): QKV, to_q / proj_in, to_out + residual, GEGLU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/ab_tiles.py --shapes qkv0,toq0,proj0,qkv1,toq1,proj1 --plans 0,8:1,9:1,2:1,3:1 --rounds 3 2>/dev/null | grep -v amdgpu
