#!/bin/bash
# c2 (batch 1) latency vs the single-launch GroupNorm threshold (C2D_GN_FUSED_HW, tuning only).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
  for hw in 256 1024 4096; do
    C2D_GN_FUSED_HW=$hw timeout -k 10 200 python -u bench.py --batch 1 --steps 4 --warmup 1 --no-cpu-baseline --no-pmc --no-configs > /tmp/b.json 2>/tmp/b.err || { tail -3 /tmp/b.err; exit 1; }
    python3 -c "import json; d=json.load(open('/tmp/b.json')); print('fused_hw=$hw', 'c2 latency %.4f s' % (1.0/d['value']))"
  done
done
