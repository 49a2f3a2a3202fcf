#!/bin/bash
# Same-box A/B of two builds of libc2d_hip.so (C2D_LIB): dominant-kernel timing and the bench, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
A=${A:-clap2diffusion_amd/libc2d_ab_old.so}; B=${B:-clap2diffusion_amd/libc2d_hip.so}
for r in 1 2; do
  for L in $A $B; do
    echo "== $L (round $r)"
    C2D_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-configs 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('img/s', d['value'], 'dom us', d['roofline']['avg_us'])" || exit 1
  done
done
