#!/bin/bash
# Round 4: d = 40 self-attention wave stagger (C2D_ATTN_STG) -- attention parity tests with it on,
# a bit-identity check against the unstaggered kernel, then same-box timings, three alternations.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention" \
  > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u - <<'PY' || exit 1
import os, subprocess, sys, torch
code = r'''
import torch, sys
from clap2diffusion_amd import ops
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
b, h, l, d = 4, 8, 4096, 40
q = torch.randn(b * l, h * d, device=dev, generator=g).half()
k = torch.randn(b * l, h * d, device=dev, generator=g).half()
v = torch.randn(b * l, h * d, device=dev, generator=g).half()
o = ops.attention(q, k, v, b, h, l, l, d)
torch.save(o.cpu(), sys.argv[1])
'''
for stg in ("0", "1"):
    subprocess.run([sys.executable, "-c", code, f"/tmp/attn_stg{stg}.pt"], check=True, env={**os.environ, "C2D_ATTN_STG": stg})
a, b = torch.load("/tmp/attn_stg0.pt"), torch.load("/tmp/attn_stg1.pt")
print("stagger vs unstaggered: bit-identical" if torch.equal(a, b) else f"DIFFER max {(a.float()-b.float()).abs().max()}")
PY
for r in 1 2 3; do
  for stg in 0 1; do
    echo "== C2D_ATTN_STG=$stg round $r"
    C2D_ATTN_STG=$stg timeout -k 10 120 python -u scripts/bench_attn.py 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
  done
done > $O/ab.txt
cat $O/ab.txt
