#!/bin/bash
# Same-box A/B of two library builds on the attention microbench (C2D_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
A=${A:-clap2diffusion_amd/libc2d_ab_old.so}; B=${B:-clap2diffusion_amd/libc2d_hip.so}
for r in 1 2; do
  for L in $B $A; do
    echo "== $L (round $r)"
    C2D_LIB=$PWD/$L timeout -k 10 200 python -u scripts/bench_attn.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
