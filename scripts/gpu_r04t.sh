#!/bin/bash
# Round 4: same-box bench A/B of the deep-ring small tiles in the pipeline (libc2d_hip_deep.so maps
# tiles 3 / 9 / 8 / 2 to their deep-ring twins 4 / 10 / 6 / 5), two alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
for r in 1 2; do
  for L in libc2d_hip libc2d_hip_deep; do
    C2D_LIB=$PWD/clap2diffusion_amd/$L.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L round $r: c3', d['value'], 'c2', d['c2_latency_s'], 'c5', d['c5_images_per_s'])" | tee -a $O/ab.txt || exit 1
  done
done
