#!/bin/bash
# Round 4: GEGLU epilogue math packed (v_pk_*_f32, default) vs scalar f32 with SLP vectorisation off
# (libc2d_hip_scal.so), and SLP off alone (libc2d_hip_noslp.so): bit-identity of the GEGLU outputs,
# per-shape timings (two alternations), then a same-box bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
for L in libc2d_hip libc2d_hip_scal libc2d_hip_noslp; do
  C2D_LIB=$PWD/clap2diffusion_amd/$L.so timeout -k 10 120 python -u - $L <<'PY' || exit 1
import sys, torch, math
sys.path.insert(0, ".")
from clap2diffusion_amd import ops
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
outs = {}
for name, (h, cin, cout, n) in {"geglu0": (64, 320, 2560, 16), "geglu1": (32, 640, 5120, 16), "geglu2": (16, 1280, 10240, 16)}.items():
    x = torch.randn(n, h, h, cin, generator=g).to(dev, torch.float16)
    w = torch.randn(cout, cin, 1, 1, generator=g) / math.sqrt(cin)
    wp, kp = ops.pack_conv_weight(w)
    b = torch.randn(cout, generator=g).to(dev) * 0.1
    outs[name] = ops.conv(x, wp.to(dev), kp, cout, ksize=1, bias=b, act="geglu").cpu()
torch.save(outs, f"gpurun_out/r04u/out_{sys.argv[1]}.pt")
PY
done
python3 - <<'PY' || exit 1
import torch
a = torch.load("gpurun_out/r04u/out_libc2d_hip.pt")
for L in ("libc2d_hip_scal", "libc2d_hip_noslp"):
    b = torch.load(f"gpurun_out/r04u/out_{L}.pt")
    for k in a:
        print(L, k, "bit-identical" if torch.equal(a[k], b[k]) else f"DIFFERS max {(a[k].float()-b[k].float()).abs().max().item()}")
PY
for r in 1 2; do
  for L in libc2d_hip libc2d_hip_scal libc2d_hip_noslp; do
    echo "== lib $L round $r" >> $O/ab.txt
    C2D_LIB=$PWD/clap2diffusion_amd/$L.so timeout -k 10 200 python -u scripts/ab_tiles.py --shapes geglu0,geglu1,geglu2,qkv0,proj0,conv0p --plans 0 --rounds 3 2>/dev/null | grep -v amdgpu >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
for r in 1 2; do
  for L in libc2d_hip libc2d_hip_scal; do
    C2D_LIB=$PWD/clap2diffusion_amd/$L.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L round $r: c3', d['value'], 'c2', d['c2_latency_s'], 'c5', d['c5_images_per_s'])" | tee -a $O/bench_ab.txt || exit 1
  done
done
