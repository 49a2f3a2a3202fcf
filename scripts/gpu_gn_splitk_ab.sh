#!/bin/bash
# A/B of the working tree (libc2d_hip.so) against the last commit (libc2d_hip_head.so):
# GroupNorm per shape (N = 2 / 16), split-K conv shapes at N = 2, c2 latency.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
  for v in new head; do
    lib=$PWD/clap2diffusion_amd/libc2d_hip.so; [ $v = head ] && lib=$PWD/clap2diffusion_amd/libc2d_hip_head.so
    for n in 2 16; do
      C2D_LIB=$lib GN_N=$n timeout -k 10 60 python -u scripts/bench_norm_graph.py 2>&1 | grep "^GN" | sed "s/^/$v N=$n /" || exit 1
    done
    for shp in "3 8 1280 1280" "3 16 2560 1280" "3 32 640 640" "3 64 960 320"; do
      C2D_LIB=$lib TAG=$v timeout -k 10 60 python -u scripts/time_gemm.py $shp --n 2 --res || exit 1
    done
    C2D_LIB=$lib timeout -k 10 200 python -u bench.py --batch 1 --steps 4 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > /tmp/b.json 2>/tmp/b.err || { tail -3 /tmp/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/b.json')); print('$v c2 latency %.4f s' % (1.0/d['value']))"
  done
done
