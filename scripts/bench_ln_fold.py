"""LayerNorm -> panel GEMM against the folded GEMM (C2D_PRO_LNFOLD), graph-replayed per call:
the UNet's norm1 -> fused QKV and norm3 -> GEGLU shapes at c3 (M = 65536; level 1: 16384 x 640),
c2 (8192), c5 (73728).

python scripts/bench_ln_fold.py [--all | --extra]"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import ops  # noqa: E402

dev = torch.device("cuda")


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    best = 1e9
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1000 / reps)
    return best


ALL = "--all" in sys.argv   # also shapes the planner keeps off the panel GEMM (the fold forces it)
SHAPES = ((65536, 320), (8192, 320), (73728, 320), (16384, 640), (2048, 640))
if "--extra" in sys.argv:   # c5's level 1 (8 x 48^2 rows) and c2's CFG-shared half batch
    SHAPES, ALL = ((18432, 640), (4096, 320)), True
for m, c in SHAPES:
    for cout, geglu in ((3 * c, False), (8 * c, True), (c, False)):
        if not (ALL or ops.panel_gemm(m, c, cout, geglu)):
            continue
        gen = torch.Generator(device="cpu").manual_seed(0)
        x = (torch.randn(m, c, generator=gen) * 2 + 5).half().to(dev)
        gamma, beta = (1 + 0.1 * torch.randn(c, generator=gen)).to(dev), (0.1 * torch.randn(c, generator=gen)).to(dev)
        w = torch.randn(cout, c, generator=gen) / math.sqrt(c)
        b = (0.1 * torch.randn(cout, generator=gen)).to(dev)
        wp, kp = ops.pack_linear_weight(w)
        wp = wp.to(dev)
        wf, bf = ops.fold_layernorm(wp, b, gamma, beta, c)
        act = "geglu" if geglu else None
        y = torch.empty(m, c, device=dev, dtype=torch.float16)
        o1 = torch.empty(m, cout // 2 if geglu else cout, device=dev, dtype=torch.float16)
        o2 = torch.empty_like(o1)

        def unfused():
            ops.layer_norm(x, gamma, beta, 1e-5, out=y)
            ops.conv(y, wp, kp, cout, ksize=1, bias=b, act=act, out=o1)

        def ln_only():
            ops.layer_norm(x, gamma, beta, 1e-5, out=y)

        def gemm_only():
            ops.conv(y, wp, kp, cout, ksize=1, bias=b, act=act, out=o1)

        def folded():
            ops.conv(x, wf, kp, cout, ksize=1, bias=bf, act=act, out=o2, ln_fold=1e-5)

        tu, tl, tg, tf = timed(unfused), timed(ln_only), timed(gemm_only), timed(folded)
        err = ((o1.float() - o2.float()).norm() / o1.float().norm()).item()
        print(f"M={m:6d} {'GEGLU' if geglu else 'plain'} {c}->{cout} (planner tile {70 if ops.panel_gemm(m, c, cout, geglu) else 'other'}): LN {tl:6.1f} + GEMM {tg:6.1f} = {tu:6.1f} us"
              f" | folded {tf:6.1f} us | rel-L2 {err:.1e}", flush=True)
