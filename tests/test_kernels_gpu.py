"""Per-kernel numerics: every HIP entry point against a plain PyTorch fp32
reference of the same op on the same (seeded) inputs.

Tolerance: fp16 storage / fp32 accumulation vs fp32 reference,
max|err| <= 2e-2 * max|ref| and rel-L2 <= 5e-3 unless a test states otherwise.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from clap2diffusion_amd import ops
from tests import parity_log

pytestmark = pytest.mark.gpu


def close(out, ref, tol_max=2e-2, tol_l2=5e-3):
    out = out.float().cpu()
    ref = ref.float().cpu()
    assert torch.isfinite(out).all(), "non-finite output"
    err = (out - ref)
    rel_l2 = (err.norm() / ref.norm().clamp_min(1e-12)).item()
    rel_max = (err.abs().max() / ref.abs().max().clamp_min(1e-12)).item()
    parity_log.record(rel_l2=rel_l2, rel_max=rel_max, tol_l2=tol_l2, tol_max=tol_max)
    assert rel_l2 <= tol_l2 and rel_max <= tol_max, f"rel_l2={rel_l2:.3e} rel_max={rel_max:.3e}"


@pytest.fixture
def force_plan():
    """Force the implicit-GEMM plan through c2d_set_plan_override for one test."""
    held = []

    def _force(tile, split):
        fp = ops.force_plan(tile, split)
        fp.__enter__()
        held.append(fp)
    yield _force
    for fp in reversed(held):   # each restores the override its __enter__ found
        fp.__exit__(None, None, None)


def gen(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


@pytest.mark.parametrize("n,h,cin,cout,stride,up", [
    (2, 16, 320, 320, 1, False),
    (2, 16, 320, 640, 2, False),
    (2, 8, 640, 640, 1, True),
    (3, 8, 1280, 1280, 1, False),
    (16, 64, 320, 320, 1, False),
    (16, 32, 640, 640, 1, False),
    (4, 32, 192, 320, 1, False),
])
def test_conv3x3(dev, n, h, cin, cout, stride, up):
    x = gen(n, cin, h, h, seed=1)
    w = gen(cout, cin, 3, 3, seed=2, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=3)
    xi = F.interpolate(x, scale_factor=2.0, mode="nearest") if up else x
    ref = F.conv2d(xi, w, b, stride=stride, padding=1)
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev), stride=stride, up=up)
    close(nchw(out), ref)


@pytest.mark.parametrize("n,h,cin,cout", [
    (16, 64, 320, 4),     # UNet conv_out at the bench shape (256x320 tile, 4 live columns)
    (2, 128, 128, 4),     # VAE conv_out shape class
    (16, 64, 320, 12),    # width not a multiple of 8: 8-byte epilogue chunks
])
def test_conv3x3_narrow_outputs(dev, n, h, cin, cout):
    x = gen(n, cin, h, h, seed=31)
    w = gen(cout, cin, 3, 3, seed=32, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=33)
    resid = gen(n, cout, h, h, seed=34)
    ref = F.conv2d(x, w, b, padding=1) + resid
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev),
                   resid=nhwc(resid).half().to(dev))
    close(nchw(out), ref)


def test_conv3x3_gn_silu_temb_resid(dev):
    n, h, cin, cout, groups = 2, 16, 320, 640, 32
    x = gen(n, cin, h, h, seed=4, scale=2.0) + 0.5
    gamma, beta = gen(cin, seed=5) * 0.2 + 1, gen(cin, seed=6) * 0.2
    w = gen(cout, cin, 3, 3, seed=7, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=8)
    temb = gen(n, cout, seed=9)
    resid = gen(n, cout, h, h, seed=10)
    ref = F.conv2d(F.silu(F.group_norm(x, groups, gamma, beta, 1e-5)), w, b, padding=1) + temb[:, :, None, None] + resid
    xd = nhwc(x).half().to(dev)
    sc, sh = ops.group_norm_stats(xd, groups, 1e-5, gamma.float().to(dev), beta.float().to(dev))
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(xd, wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev), gn=(sc, sh), gn_silu=True,
                   temb=temb.half().to(dev), resid=nhwc(resid).half().to(dev))
    close(nchw(out), ref)


@pytest.mark.parametrize("n,h,c0,c1,cout,act", [
    (16, 8, 1280, 0, 1280, None),       # L3 resnet conv: 80 tiles -> split-K
    (16, 8, 1280, 1280, 1280, None),    # L3 up-block conv over the skip concat (K = 23040)
    (16, 16, 1280, 0, 1280, "silu"),    # L2 conv with an activation through the combine kernel
])
def test_conv3x3_split_k_epilogue(dev, n, h, c0, c1, cout, act):
    """Under-filled levels split K over blocks (fp32 slabs + combine kernel that
    applies bias -> act -> +temb -> +resid); same numerics bar as the direct path."""
    from clap2diffusion_amd import _lib
    import ctypes
    d = _lib.ConvDesc()
    d.c0, d.c1, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride = c0, c1, n, h, h, h, h, 3, 1
    d.cout, d.kpad = cout, ops.kpad_of(9 * (c0 + c1))
    assert _lib.lib().c2d_conv2d_igemm_workspace_size(ctypes.byref(d)) > 0, "shape expected to split K"
    cin = c0 + c1
    x = gen(n, cin, h, h, seed=21)
    w = gen(cout, cin, 3, 3, seed=22, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=23)
    temb = gen(n, cout, seed=24) if act is None else None
    resid = gen(n, cout, h, h, seed=25)
    ref = F.conv2d(x, w, b, padding=1)
    if act == "silu":
        ref = F.silu(ref)
    if temb is not None:
        ref = ref + temb[:, :, None, None]
    ref = ref + resid
    xd = nhwc(x).half().to(dev)
    x0, x1 = (xd[..., :c0].contiguous(), xd[..., c0:].contiguous()) if c1 else (xd, None)
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(x0, wp.to(dev), kp, cout, ksize=3, x2=x1, bias=b.float().to(dev), act=act,
                   temb=None if temb is None else temb.half().to(dev), resid=nhwc(resid).half().to(dev))
    close(nchw(out), ref)


# every tile configuration left in igemm.hip's kDmaTiles, forced through
# c2d_set_plan_override and confirmed through c2d_conv2d_igemm_plan
DMA_TILE_IDS = [25, 40, 41, 28, 29, 7, 1, 2, 3, 8, 9, 80, 81]


@pytest.mark.parametrize("tile", DMA_TILE_IDS)
@pytest.mark.parametrize("k,split", [(3, 1), (1, 1), (3, 2)])
def test_every_dma_tile_forced(dev, force_plan, tile, k, split):
    n, h, cin, cout = 4, 16, 320, 640
    force_plan(tile, split)
    x = gen(n, cin, h, h, seed=91)
    w = gen(cout, cin, k, k, seed=92, scale=1.0 / math.sqrt(k * k * cin))
    b = gen(cout, seed=93)
    resid = gen(n, cout, h, h, seed=94)
    ref = F.conv2d(x, w, b, padding=k // 2) + resid
    wp, kp = ops.pack_conv_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=k, bias=b.float().to(dev),
                       resid=nhwc(resid).half().to(dev))
    assert plans == [(tile, split)], plans
    close(nchw(out), ref)


@pytest.mark.parametrize("split,ran", [(2, 2), (3, 3), (4, 4), (6, 6), (8, 8), (12, 12), (16, 15)])
def test_split_k_combine_every_count(dev, force_plan, split, ran):
    """splitk_reduce_kernel at every slice count the planner produces: the unrolled
    compile-time counts (2, 3, 4, 6, 8, 12) and the generic loop (16 on K = 180 steps runs
    15 slices of 12), with bias + time embedding + residual."""
    n, h, cin, cout = 2, 16, 1280, 640
    force_plan(7, split)
    x = gen(n, cin, h, h, seed=81)
    w = gen(cout, cin, 3, 3, seed=82, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=83)
    temb = gen(n, cout, seed=84)
    resid = gen(n, cout, h, h, seed=85)
    ref = F.conv2d(x, w, b, padding=1) + temb[:, :, None, None] + resid
    wp, kp = ops.pack_conv_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev),
                       temb=temb.half().to(dev), resid=nhwc(resid).half().to(dev))
    assert plans == [(7, ran)], plans
    close(nchw(out), ref)


@pytest.mark.parametrize("n,h,cin,cout,tile,split", [
    (16, 16, 1280, 1280, 0, 0),    # c3's L2 resnet conv at its planned split
    (16, 8, 1280, 1280, 0, 0),     # c3's L3 conv (planned split)
    (2, 16, 1280, 640, 7, 4),      # forced split 4 on the 128x320 DMA tile
    (2, 8, 1280, 1280, 41, 16),    # forced split 16 on the ping-pong 256x256 tile
])
def test_split_k_cancelling_partials_beyond_fp16(dev, force_plan, n, h, cin, cout, tile, split):
    """K slices whose partial sums cancel: channels [0, cin/2) carry weights +B, the rest -B,
    on inputs offset by +A, so each slice's partial is ~A*B*9*(channels per slice) (> 65504,
    beyond fp16) while the output -- the sum over all slices -- stays ~1e3 and fits fp16.  The
    combine must give the single-pass result (fp32 partials; fp16 partials overflow to inf
    here, or lose 2^-11 of a partial's magnitude)."""
    if tile:
        force_plan(tile, split)
    A, B = 16.0, 10.0
    sgn = torch.ones(cin)
    sgn[cin // 2:] = -1.0
    x = (gen(n, cin, h, h, seed=61) + A).half().float()
    w = (gen(cout, cin, 3, 3, seed=62, scale=0.05) + B * sgn[None, :, None, None]).half().float()
    b = gen(cout, seed=63)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).float()
    assert ref.abs().max() < 3e4, "output must fit fp16"
    wp, kp = ops.pack_conv_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev))
    assert plans and plans[0][1] > 1, f"shape expected to split K: {plans}"
    close(nchw(out), ref, tol_max=5e-3, tol_l2=2e-3)


@pytest.mark.parametrize("n,h,w,c0,c1,silu", [
    (2, 16, 24, 320, 0, True),      # non-square, the small-image path's shapes
    (16, 64, 64, 320, 0, True),     # c3's level-0 norm1 / norm2
    (2, 64, 64, 640, 320, True),    # an up block's norm1 over the skip concat
    (3, 8, 8, 1280, 0, False),
])
def test_groupnorm_pad(dev, n, h, w, c0, c1, silu):
    """c2d_groupnorm_pad: act(GroupNorm(cat[x, x2])) written zero-bordered, [n][h+2][w+2][c]."""
    c = c0 + c1
    x = gen(n, c, h, w, seed=141, scale=2.0) + 0.3
    gamma, beta = gen(c, seed=142) * 0.2 + 1, gen(c, seed=143) * 0.2
    xd = nhwc(x).half()
    ref = F.group_norm(nchw(xd.float()), 32, gamma, beta, 1e-5)
    if silu:
        ref = F.silu(ref)
    ref = F.pad(ref, (1, 1, 1, 1))
    xd = xd.to(dev)
    x0, x1 = (xd[..., :c0].contiguous(), xd[..., c0:].contiguous()) if c1 else (xd, None)
    out = ops.group_norm(x0, 32, 1e-5, gamma.to(dev), beta.to(dev), silu, x2=x1, pad=True)
    assert out.shape == (n, h + 2, w + 2, c)
    o = out.float().cpu()
    border = torch.ones(h + 2, w + 2, dtype=torch.bool)
    border[1:-1, 1:-1] = False
    assert (o[:, border] == 0).all(), "border pixels must be exact zeros"
    close(nchw(o), ref)


@pytest.mark.parametrize("n,h,cin,cout,tile,split,form", [
    (16, 64, 320, 320, 0, 0, "resid"),    # c3's level-0 conv2: the planner's tile 42
    (16, 64, 640, 320, 0, 0, "temb"),     # an up block's conv1 over the concat (GN'd into one padded source)
    (4, 64, 320, 320, 42, 1, "plain"),    # forced tile 42 on a 64-tile grid
    (4, 64, 320, 640, 42, 5, "resid"),    # forced split: one channel block per slice
    (4, 64, 960, 320, 42, 4, "temb"),     # 15 channel blocks in 4 slices (4, 4, 4, 3)
    (2, 32, 640, 320, 0, 0, "resid"),     # other tiles over the padded source (a valid 3x3)
    (2, 32, 320, 640, 0, 0, "resid"),     # c2's level-1 first conv1: the measured table's (43, 5)
    (2, 16, 1280, 1280, 0, 0, "temb"),    # c2's level-2 convs: (44, 10)
    (3, 8, 640, 320, 7, 2, "plain"),
    (16, 32, 640, 640, 0, 0, "resid"),    # c3's level-1 conv2: the planner's tile 43 (width 32), no split
    (16, 32, 960, 640, 0, 0, "temb"),     # a level-1 up block's conv1 over the padded concat (15 channel blocks)
    (16, 16, 640, 1280, 0, 0, "temb"),    # c3's level-2 first conv1: tile 44 (width 16), 2 K slices
    (2, 32, 320, 640, 43, 1, "plain"),    # forced tile 43 on a small grid
    (2, 32, 640, 320, 43, 3, "temb"),     # forced split: 10 channel blocks in 3 slices (4, 4, 2)
    (1, 16, 960, 320, 44, 1, "resid"),    # forced tile 44, one image (two 8-row tiles)
    (2, 16, 640, 640, 44, 4, "plain"),    # tile 44 with 4 slices of whole channel blocks
])
def test_conv3x3_padded_source(dev, force_plan, n, h, cin, cout, tile, split, form):
    """3x3 conv over a zero-bordered source (c2d_conv_desc::src_pad): the row-ring tiles 42 / 43 / 44
    (igemm_pp16r.h: the padded image rows of a channel block staged once into a ring of LDS row
    slots, taps as row-shifted fragment reads; output width 64 / 32 / 16) and every other tile as a
    valid 3x3 over the padded image."""
    x = gen(n, cin, h, h, seed=151)
    w = gen(cout, cin, 3, 3, seed=152, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=153)
    ref = F.conv2d(x, w, b, padding=1)
    temb = resid = None
    if form == "temb":
        temb = gen(n, cout, seed=154)
        ref = ref + temb[:, :, None, None]
    if form == "resid":
        resid = gen(n, cout, h, h, seed=155)
        ref = ref + resid
    xp = torch.zeros(n, h + 2, h + 2, cin)
    xp[:, 1:-1, 1:-1] = nhwc(x)
    if tile:
        force_plan(tile, split)
    wp, kp = ops.pack_conv_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(xp.half().to(dev), wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev), padded=True,
                       temb=None if temb is None else temb.half().to(dev),
                       resid=None if resid is None else nhwc(resid).half().to(dev))
    assert out.shape == (n, h, h, cout)
    rr = {64: 42, 32: 43, 16: 44}
    rr_any = (42, 43, 44)
    # the row ring at c3's batch (N = 16) and on the N = 2 shapes of the measured table (kRrHints:
    # every c2 ResnetBlock2D 3x3 at levels 0-2 but the level-0 320 -> 320)
    c2_rr = {(64, 640, 320), (64, 960, 320), (32, 320, 640), (32, 640, 640), (32, 960, 640), (32, 1280, 640),
             (32, 1920, 640), (16, 640, 1280), (16, 1280, 1280), (16, 1920, 1280), (16, 2560, 1280)}
    want_rr = h in rr and (n == 16 or (n == 2 and (h, cin, cout) in c2_rr))
    if tile:
        assert plans == [(tile, split)], plans
    elif want_rr:
        assert plans[0][0] == rr[h], plans
    else:
        assert plans[0][0] not in rr_any, plans
    if not tile:
        assert ops.rowring_conv(n, h, h, cin, cout) == want_rr
    if not tile and n == 16:   # the planner keeps the split 256-row tile where the row ring loses
        long_k = {32: 1920, 16: 1280}.get(h)
        if long_k:
            assert not ops.rowring_conv(n, h, h, long_k, cout)
    close(nchw(out), ref)


@pytest.mark.parametrize("n,h,w,cin,cout,act,bias", [
    (3, 61, 61, 320, 2560, "geglu", True),    # K = 320 (5 K steps), 590 tiles: several per workgroup, ragged M
    (16, 64, 64, 320, 960, None, False),      # the L0 QKV shape, 342 x 4 tiles, no bias
    (4, 37, 41, 640, 1280, None, True),       # K = 640, 160 tiles (< one per CU), ragged M
    (2, 50, 50, 1280, 2560, "geglu", True),   # K = 1280 (20 K steps), 270 tiles
    (1, 9, 7, 320, 768, None, True),          # a single partial tile
])
def test_persistent_carried_epilogue_gemm(dev, force_plan, n, h, w, cin, cout, act, bias):
    """Tile 50 (igemm_pps.h): the persistent 192 x 256 ping-pong 1x1 GEMM whose epilogue
    (bias, GEGLU h * gelu(g), fp16 stores) rides in the next tile's K loop, against torch fp32
    (GEGLU with the exact erf GELU: the kernel's sigmoid-form GELU is within 3.4e-5)."""
    force_plan(50, 0)
    x = gen(n, cin, h, w, seed=131)
    wt = gen(cout, cin, 1, 1, seed=132, scale=1.0 / math.sqrt(cin))
    b = gen(cout, seed=133) if bias else None
    ref = F.conv2d(x, wt, b)
    wp, kp = ops.pack_conv_weight(wt)
    bd = b.float().to(dev) if bias else None
    if act == "geglu":
        wi, bi = ops.geglu_interleave(wt[:, :, 0, 0], b)
        wp, kp = ops.pack_linear_weight(wi)
        bd = bi.float().to(dev) if bias else None
        hh, gg = ref.chunk(2, dim=1)
        ref = hh * F.gelu(gg)
    with ops.record_conv_plans() as plans:
        out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=1, bias=bd, act=act)
    assert plans == [(50, 1)], plans
    close(nchw(out), ref)


@pytest.mark.parametrize("tile", DMA_TILE_IDS)
@pytest.mark.parametrize("cout,temb,resid,bias", [
    (336, True, True, True),     # 16-B (W = 8) form, every operand, ragged last column tile
    (332, True, True, True),     # 8-B (W = 4) generic form (cout % 8 != 0)
    (320, False, True, False),   # residual without a bias (zero bias in the image write)
    (320, True, False, True),    # time embedding alone
])
def test_epilogue_operand_forms(dev, force_plan, tile, cout, temb, resid, bias):
    """The epilogue forms (epilogue.h: workgroup image on the ping-pong tiles, per-wave
    prefetch on the 16x16 DMA family, compact / plain loops) on a ragged M (2 x 13 x 17
    pixels: partial row tiles, rows straddling images) against torch fp32."""
    n, h, w_, cin = 2, 13, 17, 320
    force_plan(tile, 1)
    x = gen(n, cin, h, w_, seed=111)
    w = gen(cout, cin, 3, 3, seed=112, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=113) if bias else None
    te = gen(n, cout, seed=114) if temb else None
    r = gen(n, cout, h, w_, seed=115) if resid else None
    ref = F.conv2d(x, w, b, padding=1)
    if te is not None:
        ref = ref + te[:, :, None, None]
    if r is not None:
        ref = ref + r
    wp, kp = ops.pack_conv_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(nhwc(x).half().to(dev), wp.to(dev), kp, cout, ksize=3,
                       bias=b.float().to(dev) if b is not None else None,
                       temb=te.half().to(dev) if te is not None else None,
                       resid=nhwc(r).half().to(dev) if r is not None else None)
    assert plans == [(tile, 1)], plans
    close(nchw(out), ref)


@pytest.mark.parametrize("tile", [t for t in DMA_TILE_IDS if t not in (7, 8, 9, 40, 80, 81)])   # odd column tiles: no GEGLU
def test_every_dma_tile_forced_geglu(dev, force_plan, tile):
    m, cin, inner = 1024, 320, 640
    force_plan(tile, 1)
    x = gen(m, cin, seed=95)
    w = gen(2 * inner, cin, seed=96, scale=1.0 / math.sqrt(cin))
    b = gen(2 * inner, seed=97)
    hh, gg = (x @ w.t() + b).chunk(2, -1)
    ref = hh * F.gelu(gg)
    wi, bi = ops.geglu_interleave(w, b)
    wp, kp = ops.pack_linear_weight(wi)
    with ops.record_conv_plans() as plans:
        out = ops.conv(x.half().to(dev), wp.to(dev), kp, 2 * inner, ksize=1, bias=bi.float().to(dev), act="geglu")
    assert plans == [(tile, 1)], plans
    close(out, ref)


# the panel GEMM (tile 70, igemm_panel.h): K = 320 / 640, 1x1, plain / residual / GEGLU; M not a
# multiple of the 128-row panel, column blocks not a multiple of the 8 waves, and the column split
# over several workgroups per panel (small M)
@pytest.mark.parametrize("m,cin,cout,res", [
    (4096, 320, 960, False),       # QKV-shaped, 30 column blocks over 8 waves
    (300, 320, 320, True),         # ragged last panel, column split, residual
    (2048, 640, 1920, False),      # K = 640 (160 KiB panel), column split
    (1000, 640, 640, True),
])
def test_panel_gemm_forced(dev, force_plan, m, cin, cout, res):
    force_plan(70, 0)
    x = gen(m, cin, seed=101)
    w = gen(cout, cin, seed=102, scale=1.0 / math.sqrt(cin))
    b = gen(cout, seed=103)
    r = gen(m, cout, seed=104) if res else None
    ref = x @ w.t() + b + (r if res else 0)
    wp, kp = ops.pack_linear_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(x.half().to(dev), wp.to(dev), kp, cout, ksize=1, bias=b.float().to(dev),
                       resid=r.half().to(dev) if res else None)
    assert plans == [(70, 1)], plans
    close(out, ref)


@pytest.mark.parametrize("m,cin,inner", [
    (2048, 320, 1280), (777, 640, 2560),
    (8100, 320, 1280),   # 64 panels x 4 column splits: 5 column blocks per wave (the carried epilogue's steady state), ragged last panel
])
def test_panel_gemm_forced_geglu(dev, force_plan, m, cin, inner):
    force_plan(70, 0)
    x = gen(m, cin, seed=105)
    w = gen(2 * inner, cin, seed=106, scale=1.0 / math.sqrt(cin))
    b = gen(2 * inner, seed=107)
    hh, gg = (x @ w.t() + b).chunk(2, -1)
    ref = hh * F.gelu(gg)
    wi, bi = ops.geglu_interleave(w, b)
    wp, kp = ops.pack_linear_weight(wi)
    with ops.record_conv_plans() as plans:
        out = ops.conv(x.half().to(dev), wp.to(dev), kp, 2 * inner, ksize=1, bias=bi.float().to(dev), act="geglu")
    assert plans == [(70, 1)], plans
    close(out, ref)


@pytest.mark.parametrize("m,c,cout,geglu,mean", [
    (4096, 320, 960, False, 0.0), (2048, 320, 2560, True, 0.0),      # fused QKV / GEGLU of level 0
    (1000, 320, 960, False, 40.0), (300, 320, 2560, True, -25.0),    # ragged last panel, |row mean| >> std
    (2048, 640, 5120, True, 0.0), (700, 640, 1920, False, 30.0),     # level 1 (the register-ring panel kernel)
])
def test_panel_gemm_layernorm_fold(dev, m, c, cout, geglu, mean):
    """LayerNorm folded into the panel GEMM (C2D_PRO_LNFOLD, igemm_panel_dma_kernel LNF: the
    LDS panel normalised in place, then W diag(gamma) with bias b + W beta) against torch's
    LayerNorm -> Linear (diffusers BasicTransformerBlock norm1 -> to_q/k/v, norm3 -> GEGLU);
    rows offset by up to +-30 on top of `mean` (|mean| >> std: the shifted second pass)."""
    x = gen(m, c, seed=110) + mean + gen(m, 1, seed=111) * 30.0
    gamma, beta = 1.0 + 0.2 * gen(c, seed=112), 0.2 * gen(c, seed=113)
    w = gen(cout, c, seed=114, scale=1.0 / math.sqrt(c))
    b = 0.1 * gen(cout, seed=115)
    xh = x.half()
    y = F.layer_norm(xh.float(), (c,), gamma, beta, 1e-5) @ w.t() + b
    if geglu:
        hh, gg = y.chunk(2, -1)
        ref = hh * F.gelu(gg)
        w, b = ops.geglu_interleave(w, b)
    else:
        ref = y
    wp, kp = ops.pack_linear_weight(w)
    wf, bf = ops.fold_layernorm(wp, b, gamma, beta, c)
    with ops.record_conv_plans() as plans:
        out = ops.conv(xh.to(dev), wf.to(dev), kp, cout, ksize=1, bias=bf.to(dev), act="geglu" if geglu else None,
                       ln_fold=1e-5)
    assert plans == [(70, 1)], plans
    close(out, ref)


def test_panel_gemm_ineligible_falls_back(dev, force_plan):
    """Forcing tile 70 on a shape it does not take (K = 1280) leaves the planner's choice."""
    force_plan(70, 0)
    x = gen(512, 1280, seed=108)
    w = gen(640, 1280, seed=109, scale=1.0 / math.sqrt(1280))
    wp, kp = ops.pack_linear_weight(w)
    with ops.record_conv_plans() as plans:
        out = ops.conv(x.half().to(dev), wp.to(dev), kp, 640, ksize=1)
    assert plans and plans[0][0] != 70, plans
    close(out, x @ w.t())


@pytest.mark.parametrize("n,h,c0,c1,cout,k", [
    (2, 8, 1280, 640, 640, 3),      # 64x64 DMA tiles
    (16, 32, 640, 320, 320, 3),     # 128x128 DMA tiles
    (16, 64, 320, 640, 320, 3),     # 256x128 DMA tiles
    (16, 64, 640, 320, 320, 1),     # shortcut 1x1 on the concat
    (2, 16, 96, 32, 128, 3),        # seam not 64-aligned -> register-staged kernel
])
def test_conv_dual_source_plain(dev, n, h, c0, c1, cout, k):
    x0, x1 = gen(n, c0, h, h, seed=31), gen(n, c1, h, h, seed=32)
    w = gen(cout, c0 + c1, k, k, seed=33, scale=1.0 / math.sqrt(k * k * (c0 + c1)))
    b = gen(cout, seed=34)
    ref = F.conv2d(torch.cat([x0, x1], 1), w, b, padding=k // 2)
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(nhwc(x0).half().to(dev), wp.to(dev), kp, cout, ksize=k, bias=b.float().to(dev),
                   x2=nhwc(x1).half().to(dev))
    close(nchw(out), ref)


def test_upsample_nearest2x(dev):
    x = gen(3, 40, 5, 7, seed=35)
    ref = F.interpolate(x, scale_factor=2.0, mode="nearest")
    out = ops.upsample_nearest2x(nhwc(x).half().to(dev))
    assert torch.equal(nchw(out).cpu(), ref.half())


def test_conv_dual_source_gn(dev):
    # skip-concat with a group straddling the seam (1280 + 640 = 1920, 60 ch/group)
    n, h, c0, c1, cout = 2, 8, 1280, 640, 640
    x0, x1 = gen(n, c0, h, h, seed=11), gen(n, c1, h, h, seed=12) * 3 + 1
    xc = torch.cat([x0, x1], 1)
    gamma, beta = gen(c0 + c1, seed=13) * 0.1 + 1, gen(c0 + c1, seed=14) * 0.1
    w = gen(cout, c0 + c1, 3, 3, seed=15, scale=1.0 / math.sqrt(9 * (c0 + c1)))
    ref = F.conv2d(F.silu(F.group_norm(xc, 32, gamma, beta, 1e-5)), w, None, padding=1)
    a, bb = nhwc(x0).half().to(dev), nhwc(x1).half().to(dev)
    sc, sh = ops.group_norm_stats(a, 32, 1e-5, gamma.float().to(dev), beta.float().to(dev), x2=bb)
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(a, wp.to(dev), kp, cout, ksize=3, x2=bb, gn=(sc, sh), gn_silu=True)
    close(nchw(out), ref)
    # 1x1 shortcut over the same concat, no prologue
    ws = gen(cout, c0 + c1, 1, 1, seed=16, scale=1.0 / math.sqrt(c0 + c1))
    ref2 = F.conv2d(xc, ws)
    wp2, kp2 = ops.pack_conv_weight(ws)
    out2 = ops.conv(a, wp2.to(dev), kp2, cout, ksize=1, x2=bb)
    close(nchw(out2), ref2)


def test_conv_in_padded(dev):
    # conv_in: 4 latent channels padded to 8 (generic 3x3 path, K = 72 -> 128)
    n, h = 2, 16
    x = gen(n, 4, h, h, seed=17)
    w = gen(320, 4, 3, 3, seed=18, scale=0.3)
    b = gen(320, seed=19)
    ref = F.conv2d(x, w, b, padding=1)
    xd = ops.latent_to_nhwc(x.float().to(dev), cpad=8, dup=False)
    wp, kp = ops.pack_conv_weight(w, cin_pad=8)
    out = ops.conv(xd, wp.to(dev), kp, 320, ksize=3, bias=b.float().to(dev))
    close(nchw(out), ref)


def test_conv_out_small_cout(dev):
    n, h = 2, 16
    x = gen(n, 320, h, h, seed=20)
    gamma, beta = torch.ones(320), torch.zeros(320)
    w = gen(4, 320, 3, 3, seed=21, scale=0.02)
    b = gen(4, seed=22)
    ref = F.conv2d(F.silu(F.group_norm(x, 32, gamma, beta, 1e-5)), w, b, padding=1)
    xd = nhwc(x).half().to(dev)
    sc, sh = ops.group_norm_stats(xd, 32, 1e-5, gamma.to(dev), beta.to(dev))
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(xd, wp.to(dev), kp, 4, ksize=3, bias=b.float().to(dev), gn=(sc, sh), gn_silu=True)
    close(nchw(out), ref)


@pytest.mark.parametrize("m,k,nout", [(300, 96, 288), (1024, 320, 960), (77, 768, 1280), (4096, 1280, 1280)])
def test_linear_ln(dev, m, k, nout):
    x = gen(m, k, seed=23) * 2 + 0.3
    gamma, beta = gen(k, seed=24) * 0.1 + 1, gen(k, seed=25) * 0.1
    w = gen(nout, k, seed=26, scale=1 / math.sqrt(k))
    b = gen(nout, seed=27)
    ref = F.linear(F.layer_norm(x, (k,), gamma, beta, 1e-5), w, b)
    xd = x.half().to(dev)
    st = ops.layer_norm_stats(xd, 1e-5)
    wp, kp = ops.pack_linear_weight(w)
    out = ops.conv(xd, wp.to(dev), kp, nout, ksize=1, bias=b.float().to(dev),
                   ln=(st, gamma.float().to(dev), beta.float().to(dev)))
    close(out, ref)
    # LayerNorm apply kernel
    y = ops.layer_norm(xd, gamma.float().to(dev), beta.float().to(dev), 1e-5)
    close(y, F.layer_norm(x, (k,), gamma, beta, 1e-5))


@pytest.mark.parametrize("act", ["gelu", "relu", "silu"])
def test_linear_act_resid(dev, act):
    m, k, nout = 256, 384, 192
    x, w, b, r = gen(m, k, seed=28), gen(nout, k, seed=29, scale=1 / math.sqrt(k)), gen(nout, seed=30), gen(m, nout, seed=31)
    fn = {"gelu": F.gelu, "relu": F.relu, "silu": F.silu}[act]
    ref = fn(F.linear(x, w, b)) + r
    wp, kp = ops.pack_linear_weight(w)
    out = ops.conv(x.half().to(dev), wp.to(dev), kp, nout, ksize=1, bias=b.float().to(dev), act=act,
                   resid=r.half().to(dev))
    close(out, ref)


def test_geglu(dev):
    m, c = 512, 320
    inner = 4 * c
    x = gen(m, c, seed=32)
    w = gen(2 * inner, c, seed=33, scale=1 / math.sqrt(c))
    b = gen(2 * inner, seed=34) * 0.1
    r = gen(m, inner, seed=35)
    hh, gg = F.linear(x, w, b).chunk(2, dim=-1)
    ref = hh * F.gelu(gg) + r
    wi, bi = ops.geglu_interleave(w, b)
    wp, kp = ops.pack_linear_weight(wi)
    out = ops.conv(x.half().to(dev), wp.to(dev), kp, 2 * inner, ksize=1, bias=bi.float().to(dev), act="geglu",
                   resid=r.half().to(dev))
    close(out, ref)


# shapes large enough for the planner's 256x320 tile (>= 192 output tiles), its
# epilogue variants (scripts/gpu_ab.sh PYTEST_K arms run these with C2D_TUNE_GEMM_LDSEPI=0 and 1);
# torch fp32 on the device is the reference
def test_m32_direct_epilogue_geglu(dev):
    m, c = 16384, 320
    inner = 4 * c
    x = gen(m, c, seed=70).to(dev)
    w = gen(2 * inner, c, seed=71, scale=1 / math.sqrt(c)).to(dev)
    b = (gen(2 * inner, seed=72) * 0.1).to(dev)
    r = gen(m, inner, seed=73).to(dev)
    xh, rh = x.half(), r.half()
    hh, gg = F.linear(xh.float(), w, b).chunk(2, dim=-1)
    ref = hh * F.gelu(gg) + rh.float()
    wi, bi = ops.geglu_interleave(w, b)
    wp, kp = ops.pack_linear_weight(wi)
    out = ops.conv(xh, wp, kp, 2 * inner, ksize=1, bias=bi.float(), act="geglu", resid=rh)
    close(out, ref)


def test_m32_direct_epilogue_conv_temb_resid(dev):
    n, h, cin, cout = 12, 64, 320, 320
    x = gen(n, cin, h, h, seed=74).to(dev)
    w = gen(cout, cin, 3, 3, seed=75, scale=1 / math.sqrt(9 * cin)).to(dev)
    b = (gen(cout, seed=76) * 0.1).to(dev)
    temb = gen(n, cout, seed=77).to(dev)
    resid = gen(n, cout, h, h, seed=78).to(dev)
    xh, th, rh = x.half(), temb.half(), resid.half()
    ref = F.conv2d(xh.float(), w, b, padding=1) + th.float()[:, :, None, None] + rh.float()
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(nhwc(xh), wp, kp, cout, ksize=3, bias=b.float(), temb=th, resid=nhwc(rh))
    close(nchw(out), ref)


def test_m32_direct_epilogue_linear_bias(dev):
    m, cin, cout = 16384, 320, 960
    x = gen(m, cin, seed=79).to(dev)
    w = gen(cout, cin, seed=80, scale=1 / math.sqrt(cin)).to(dev)
    b = (gen(cout, seed=81) * 0.1).to(dev)
    ref = F.linear(x.half().float(), w, b)
    wp, kp = ops.pack_linear_weight(w)
    out = ops.conv(x.half(), wp, kp, cout, ksize=1, bias=b.float())
    close(out, ref)


def test_silu_prologue(dev):
    x = gen(16, 1280, seed=36)
    w = gen(2560, 1280, seed=37, scale=1 / math.sqrt(1280))
    ref = F.linear(F.silu(x), w)
    wp, kp = ops.pack_linear_weight(w)
    out = ops.conv(x.half().to(dev), wp.to(dev), kp, 2560, ksize=1, silu_in=True)
    close(out, ref)


def attn_ref(q, k, v, b, h, lq, lk, d):
    qh = q.view(b, lq, h, d).transpose(1, 2)
    kh = k.view(b, lk, h, d).transpose(1, 2)
    vh = v.view(b, lk, h, d).transpose(1, 2)
    o = F.scaled_dot_product_attention(qh, kh, vh)
    return o.transpose(1, 2).reshape(b * lq, h * d)


@pytest.mark.parametrize("b,h,lq,lk,d", [
    (2, 8, 256, 256, 40), (2, 8, 200, 77, 40), (2, 8, 1024, 1024, 80), (2, 8, 64, 64, 160),
    (1, 8, 256, 77, 160), (2, 4, 300, 300, 64), (2, 8, 4096, 4096, 40),
    (1, 8, 9216, 9216, 40), (1, 8, 2304, 2304, 80),   # c5: 768^2 images (96^2 latent) levels 0 / 1
    # resident-K/V path (lk <= 128): several query blocks per workgroup, ragged last block
    (16, 8, 4000, 77, 40), (16, 8, 1024, 77, 80), (16, 8, 256, 77, 160), (4, 8, 700, 128, 40), (3, 8, 300, 64, 80),
])
def test_attention(dev, b, h, lq, lk, d):
    c = h * d
    qkv = gen(b * lq, 3 * c, seed=38)
    kv = gen(b * lk, 2 * c, seed=39)
    q = qkv[:, :c]
    k, v = kv[:, :c], kv[:, c:]
    ref = attn_ref(q, k, v, b, h, lq, lk, d)
    qd, kvd = qkv.half().to(dev), kv.half().to(dev)
    out = ops.attention(qd[:, :c], kvd[:, :c], kvd[:, c:], b, h, lq, lk, d)
    close(out, ref)


def test_attention_spike(dev):
    # force the online-softmax rescale: one key dominates late in the sequence
    b, h, l, d = 1, 8, 512, 40
    q = gen(b * l, h * d, seed=40)
    k = gen(b * l, h * d, seed=41)
    v = gen(b * l, h * d, seed=42)
    k[450] = q[3] * 4.0
    ref = attn_ref(q, k, v, b, h, l, l, d)
    out = ops.attention(q.half().to(dev), k.half().to(dev), v.half().to(dev), b, h, l, l, d)
    close(out, ref)


@pytest.mark.parametrize("b,h,lq,lk,d,form", [
    (2, 8, 300, 77, 40, "per_image"),     # cross-attention with a key-padding mask (resident K/V)
    (2, 8, 256, 77, 160, "per_head"),
    (1, 8, 1024, 1024, 80, "broadcast"),  # self-attention, streaming K/V
    (2, 4, 200, 333, 40, "per_image"),
])
def test_attention_key_bias(dev, b, h, lq, lk, d, form):
    q, k, v = gen(b * lq, h * d, seed=61), gen(b * lk, h * d, seed=62), gen(b * lk, h * d, seed=63)
    g = torch.Generator().manual_seed(64)
    if form == "per_image":
        bias = torch.zeros(b, 1, lk)
        for i in range(b):
            bias[i, 0, (17 + 29 * i) % lk:] = -10000.0
    elif form == "per_head":
        bias = torch.randn(b, h, lk, generator=g) * 2.0
    else:
        bias = torch.randn(1, 1, lk, generator=g)
    qh = q.view(b, lq, h, d).transpose(1, 2)
    kh = k.view(b, lk, h, d).transpose(1, 2)
    vh = v.view(b, lk, h, d).transpose(1, 2)
    ref = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=bias[:, :, None, :]).transpose(1, 2).reshape(b * lq, h * d)
    out = ops.attention(q.half().to(dev), k.half().to(dev), v.half().to(dev), b, h, lq, lk, d,
                        key_bias=bias.to(dev))
    close(out, ref)


@pytest.mark.parametrize("b,h,lq,lk,d,form", [
    (2, 8, 300, 77, 40, "per_query"),       # [B, H, Lq, Lk] (resident K/V), ragged query tail
    (1, 8, 200, 77, 80, "bh_flat"),         # [1, 1, Lq, Lk] broadcast over images and heads
    (2, 4, 256, 333, 160, "per_query"),     # streaming K/V, masked key tail
    (2, 8, 300, 77, 40, "neg_inf"),         # SDPA-style -inf entries, every row keeps a finite score
])
def test_attention_query_mask(dev, b, h, lq, lk, d, form):
    """c2d_attention_fwd_mask: an attention_mask varying over queries, as the reference
    processor hands it to get_attention_scores (models/audio_attention_processor.py:129)."""
    q, k, v = gen(b * lq, h * d, seed=71), gen(b * lk, h * d, seed=72), gen(b * lk, h * d, seed=73)
    g = torch.Generator().manual_seed(74)
    if form == "bh_flat":
        bias = torch.randn(1, 1, lq, lk, generator=g) * 3.0
    else:
        bias = torch.randn(b, h, lq, lk, generator=g) * 2.0
    if form == "neg_inf":
        drop = torch.rand(b, h, lq, lk, generator=g) < 0.4
        drop[..., 5] = False
        bias = bias.masked_fill(drop, float("-inf"))
    qh = q.view(b, lq, h, d).transpose(1, 2)
    kh = k.view(b, lk, h, d).transpose(1, 2)
    vh = v.view(b, lk, h, d).transpose(1, 2)
    ref = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=bias).transpose(1, 2).reshape(b * lq, h * d)
    out = ops.attention(q.half().to(dev), k.half().to(dev), v.half().to(dev), b, h, lq, lk, d,
                        key_bias=bias.to(dev))
    close(out, ref)


@pytest.mark.parametrize("lk", [77, 128, 200])
@pytest.mark.parametrize("d", [40, 80])
def test_attention_fully_masked_rows(dev, lk, d):
    """Rows with no finite score, against torch softmax(q.k * scale + mask) @ v in float64:
    all finfo.min -> the uniform average of V; all -inf -> NaN; -inf mixed with finfo.min ->
    uniform over the finfo.min keys; a single finite key -> that key's V.  lk = 77 / 128: the
    resident-K/V form (77 with a padded tail tile), 200: the streaming form."""
    b, h, lq = 2, 2, 40
    q, k, v = gen(b * lq, h * d, seed=171), gen(b * lk, h * d, seed=172), gen(b * lk, h * d, seed=173)
    g = torch.Generator().manual_seed(174)
    bias = torch.randn(b, h, lq, lk, generator=g) * 2.0
    fmin, ninf = torch.finfo(torch.float32).min, float("-inf")
    bias[0, 0, 3, :] = fmin
    bias[1, 1, 7, :] = ninf
    bias[0, 1, 9, :lk // 2] = ninf
    bias[0, 1, 9, lk // 2:] = fmin
    bias[1, 0, 11, :] = ninf
    bias[1, 0, 11, lk - 1] = 0.0
    bias[1, 0, 12, :] = fmin
    bias[1, 0, 12, 0] = -5.0
    q16, k16, v16 = q.half().float(), k.half().float(), v.half().float()
    qh = q16.view(b, lq, h, d).transpose(1, 2).double()
    kh = k16.view(b, lk, h, d).transpose(1, 2).double()
    vh = v16.view(b, lk, h, d).transpose(1, 2).double()
    sc = (qh @ kh.transpose(-1, -2)) / math.sqrt(d) + bias.double()
    ref = (torch.softmax(sc, -1) @ vh).transpose(1, 2).reshape(b * lq, h * d).float()
    out = ops.attention(q.half().to(dev), k.half().to(dev), v.half().to(dev), b, h, lq, lk, d,
                        key_bias=bias.to(dev)).float().cpu()
    nan_ref = torch.isnan(ref)
    assert nan_ref.view(b, lq, h, d)[1, 7, 1].all() and nan_ref.sum() == d, "torch: only the all -inf row is NaN"
    assert torch.equal(torch.isnan(out), nan_ref), "NaN exactly where torch's softmax gives NaN"
    uni = vh[0, 0].mean(0).float()
    assert torch.allclose(out.view(b, lq, h, d)[0, 3, 0], uni, atol=2e-3), "finfo.min row: mean of V"
    close(out[~nan_ref].view(-1), ref[~nan_ref].view(-1))


@pytest.mark.parametrize("d", [40, 80, 160])
def test_attention_wide_scores(dev, d):
    # scores of std ~12 (log2 units ~17): the first key tile rebases the running max
    # and later tiles rescale often; ragged lk exercises the masked tail tile
    b, h, lq, lk = 1, 4, 192, 333
    q = gen(b * lq, h * d, seed=44) * 12.0
    k = gen(b * lk, h * d, seed=45)
    v = gen(b * lk, h * d, seed=46)
    k[5] -= 3.0  # a strongly negative early key
    ref = attn_ref(q, k, v, b, h, lq, lk, d)
    out = ops.attention(q.half().to(dev), k.half().to(dev), v.half().to(dev), b, h, lq, lk, d)
    close(out, ref)


@pytest.mark.parametrize("b,h,lq,lk,scale", [
    (4, 8, 2000, 256, 1.0), (4, 8, 1800, 320, 12.0), (4, 8, 2040, 1024, 4.0),   # 8-wave blocks (>= 256 of them)
    (2, 4, 300, 256, 1.0), (2, 4, 520, 1024, 4.0),                            # small grids: 4-wave NEGC blocks
])
def test_attention_d40_w8(dev, b, h, lq, lk, scale):
    """The 8-wave d = 40 kernel (lk % 64 == 0, lk >= 256, no mask, a grid of >= 256 such blocks) and its 4-wave
    twin below that: a ragged last query block, and scores of std ~12 / ~4 so the first tile rebases the
    running max and later tiles rescale (the lazy 2^8 test)."""
    d = 40
    q = gen(b * lq, h * d, seed=47) * scale
    k = gen(b * lk, h * d, seed=48)
    v = gen(b * lk, h * d, seed=49)
    k[7] -= 3.0
    ref = attn_ref(q, k, v, b, h, lq, lk, d)
    out = ops.attention(q.half().to(dev), k.half().to(dev), v.half().to(dev), b, h, lq, lk, d)
    close(out, ref)


def test_groupnorm_stats_large_mean(dev):
    n, c, hw = 2, 640, 1024
    x = gen(n, c, 32, 32, seed=43) + 30.0
    gamma, beta = torch.ones(c), torch.zeros(c)
    ref = F.group_norm(x, 32, gamma, beta, 1e-6)
    xd = nhwc(x).half().to(dev)
    sc, sh = ops.group_norm_stats(xd, 32, 1e-6, gamma.to(dev), beta.to(dev))
    y = xd.float() * sc.view(n, 1, 1, c) + sh.view(n, 1, 1, c)
    # reference uses the fp16-rounded input for a fair statistic comparison
    ref16 = F.group_norm(nchw(xd.float().cpu()), 32, gamma, beta, 1e-6)
    close(nchw(y), ref16, tol_max=5e-3, tol_l2=1e-3)
    close(nchw(y), ref, tol_max=5e-2, tol_l2=2e-2)


def test_cfg_ddim(dev):
    b = 2
    x = gen(b, 4, 8, 8, seed=44)
    eps = gen(2 * b, 4, 8, 8, seed=45)
    coef = torch.tensor([[0.3, 0.5], [0.5, 0.7]], dtype=torch.float32)
    g = 7.5
    e = eps[:b] + g * (eps[b:] - eps[:b])
    a_t, a_p = coef[1]
    x0 = (x - (1 - a_t).sqrt() * e) / a_t.sqrt()
    ref = a_p.sqrt() * x0 + (1 - a_p).sqrt() * e
    xd = x.to(dev).contiguous()
    st = torch.tensor([1], dtype=torch.int32, device=dev)
    ops.cfg_ddim_step(nhwc(eps).half().to(dev), xd, g, coef.to(dev), st, advance=True)
    # eps was rounded to fp16 on upload
    e16 = eps.half().float()
    e = e16[:b] + g * (e16[b:] - e16[:b])
    x0 = (x - (1 - a_t).sqrt() * e) / a_t.sqrt()
    ref = a_p.sqrt() * x0 + (1 - a_p).sqrt() * e
    close(xd, ref, tol_max=1e-5, tol_l2=1e-6)
    assert st.item() == 2


def test_timestep_embedding(dev):
    ts = torch.tensor([981.0, 1.0, 500.0])
    half = 160
    freqs = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32) / half)
    for i, t in enumerate(ts):
        idx = torch.tensor([i], dtype=torch.int32, device=dev)
        out = ops.timestep_embedding(ts.to(dev), idx, 2, 320)
        a = t * freqs
        ref = torch.cat([torch.cos(a), torch.sin(a)]).expand(2, -1)
        close(out, ref, tol_max=2e-3, tol_l2=2e-3)


@pytest.mark.parametrize("silu", [True, False])
def test_groupnorm_apply_dual_source(dev, silu):
    n, h, c0, c1 = 2, 16, 640, 320
    x0, x1 = gen(n, c0, h, h, seed=50) + 1.0, gen(n, c1, h, h, seed=51) * 2
    xc = torch.cat([x0, x1], 1)
    gamma, beta = gen(c0 + c1, seed=52) * 0.1 + 1, gen(c0 + c1, seed=53) * 0.1
    ref = F.group_norm(xc, 32, gamma, beta, 1e-5)
    if silu:
        ref = F.silu(ref)
    a, b = nhwc(x0).half().to(dev), nhwc(x1).half().to(dev)
    gn = ops.group_norm_stats(a, 32, 1e-5, gamma.float().to(dev), beta.float().to(dev), x2=b)
    out = ops.group_norm_apply(a, gn, silu, x2=b)
    close(nchw(out), ref)


def test_groupnorm_deterministic(dev):
    x = nhwc(gen(4, 320, 32, 32, seed=54)).half().to(dev)
    g, b = torch.ones(320, device=dev), torch.zeros(320, device=dev)
    r = [ops.group_norm_stats(x, 32, 1e-5, g, b)[0] for _ in range(3)]
    assert all(torch.equal(r[0], t) for t in r[1:])


# c2d_groupnorm: the single-kernel path (hw <= 256) and the stats + apply
# pipeline, one- and two-source inputs, the UNet's channel / group shapes
@pytest.mark.parametrize("n,h,c0,c1,groups,silu,eps", [
    (2, 8, 1280, 0, 32, True, 1e-5),       # level-3 resnet norm (cpg 40)
    (2, 8, 1280, 1280, 32, True, 1e-5),    # level-3 up-block concat (cpg 80)
    (2, 16, 640, 320, 32, False, 1e-6),    # concat seam inside a group (cpg 30)
    (4, 16, 320, 0, 32, True, 1e-5),       # cpg 10
    (3, 16, 128, 0, 32, True, 1e-6),       # VAE-style cpg 4
    (2, 32, 640, 0, 32, True, 1e-5),       # 32^2: stats + apply pipeline
    (16, 64, 320, 0, 32, True, 1e-5),      # level-0 shape: stats + apply pipeline
    (1, 32, 1280, 1280, 32, True, 1e-5),   # 2560 channels, two sources (wide form: 10 lanes, five phases)
    (2, 32, 320, 0, 16, False, 1e-5),      # 16 groups (cpg 20) through the pipeline
    (2, 48, 640, 0, 64, True, 1e-6),       # 64 groups: two passes of the group-moment fold
    (2, 64, 320, 0, 32, True, 1e-5),       # c2's level 0 (N <= 2: the 1024-thread single launch)
    (2, 64, 640, 320, 32, True, 1e-5),     # c2's level-0 up-block concat (cpg 30, seam in a group)
    (1, 64, 960, 0, 32, False, 1e-6),      # 15 lanes per pixel row (cpg 30): four reduction phases
])
def test_groupnorm_one_call(dev, n, h, c0, c1, groups, silu, eps):
    x0 = gen(n, c0, h, h, seed=60) + 0.5
    x1 = gen(n, c1, h, h, seed=61) * 2 if c1 else None
    xc = torch.cat([x0, x1], 1) if c1 else x0
    c = c0 + c1
    gamma, beta = gen(c, seed=62) * 0.1 + 1, gen(c, seed=63) * 0.1
    a = nhwc(x0).half().to(dev)
    b = nhwc(x1).half().to(dev) if c1 else None
    # reference on the fp16-rounded input
    ref = F.group_norm(torch.cat([nchw(a.float().cpu())] + ([nchw(b.float().cpu())] if c1 else []), 1),
                       groups, gamma, beta, eps)
    if silu:
        ref = F.silu(ref)
    out = ops.group_norm(a, groups, eps, gamma.float().to(dev), beta.float().to(dev), silu, x2=b)
    close(nchw(out), ref, tol_max=5e-3, tol_l2=1e-3)
    again = ops.group_norm(a, groups, eps, gamma.float().to(dev), beta.float().to(dev), silu, x2=b)
    assert torch.equal(out, again)


# Quantisation tail (igemm.hip tail_images): c5's level-0 convs plan one K slice on 288 tiles of
# 256 x 320, so the first 7 images run that plan and the 8th its own -- every per-image pointer of
# the tail launch (both sources, the time embedding, the residual, the output; the zero-bordered
# source) is offset by 7 images.  Same numerics bar as every conv.
@pytest.mark.parametrize("c0,c1,res,tmb,padded", [
    (320, 0, True, False, False),     # ResnetBlock2D conv2 + residual
    (320, 320, False, True, False),   # up-block conv1 over the skip concat + time embedding
    (640, 320, True, True, False),    # 960 -> 320 with both epilogue terms
    (320, 0, True, True, True),       # zero-bordered source
])
def test_conv_quantisation_tail(dev, c0, c1, res, tmb, padded):
    n, h, cout = 8, 96, 320
    cin = c0 + c1
    assert ops.rowring_conv(n, h, h, cin, cout) is False
    x = gen(n, cin, h, h, seed=171)
    w = gen(cout, cin, 3, 3, seed=172, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=173)
    r = gen(n, cout, h, h, seed=174) if res else None
    te = gen(n, cout, seed=175) if tmb else None
    ref = F.conv2d(x.half().float(), w, b, padding=1)
    if te is not None:
        ref = ref + te.half().float()[:, :, None, None]
    if r is not None:
        ref = ref + r.half().float()
    wp, kp = ops.pack_conv_weight(w)
    xd = nhwc(x).half().to(dev)
    kw = dict(bias=b.float().to(dev), resid=nhwc(r).half().to(dev) if res else None,
              temb=te.half().to(dev) if tmb else None)
    with ops.record_conv_plans() as plans:
        if padded:
            xp = F.pad(xd.permute(0, 3, 1, 2), (1, 1, 1, 1)).permute(0, 2, 3, 1).contiguous()
            out = ops.conv(xp, wp.to(dev), kp, cout, ksize=3, padded=True, **kw)
        else:
            x0, x1 = (xd[..., :c0].contiguous(), xd[..., c0:].contiguous()) if c1 else (xd, None)
            out = ops.conv(x0, wp.to(dev), kp, cout, ksize=3, x2=x1, **kw)
    assert plans == [(40, 1)], plans
    if c1:   # the tail image's own plan splits K 3 ways into the workspace the call allocated
        assert ops.conv_workspace_bytes(n, h, h, c0, c1, cout, 3) == 3 * h * h * cout * 4
    close(nchw(out), ref)


# c2d_groupnorm / c2d_groupnorm_pad above 256 pixels: per-group partial pairs, then an apply
# kernel that folds them itself (two launches).  Against the three-launch API (c2d_groupnorm_stats
# -> per-channel partials + finalize, then c2d_groupnorm_apply: same per-thread moments, another
# fixed fold order) the outputs agree to the fp16 rounding of the result.
@pytest.mark.parametrize("n,h,w,c0,c1,groups,silu", [
    (2, 64, 64, 320, 0, 32, True),        # c2 level 0
    (16, 64, 64, 320, 0, 32, True),       # c3 level 0
    (2, 32, 32, 640, 320, 32, False),     # concat seam inside a group
    (3, 17, 23, 2560, 1280, 32, True),    # ragged image, two channel chunks per thread
    (5, 20, 20, 320, 0, 64, False),       # 64 groups, cpg 5
])
def test_groupnorm_two_launch_matches_three(dev, n, h, w, c0, c1, groups, silu):
    c = c0 + c1
    x0 = gen(n, c0, h, w, seed=70) * 1.5 + 0.7
    x1 = gen(n, c1, h, w, seed=71) * 3 - 1 if c1 else None
    gamma, beta = (gen(c, seed=72) * 0.1 + 1).to(dev), (gen(c, seed=73) * 0.1).to(dev)
    a = nhwc(x0).half().to(dev)
    b = nhwc(x1).half().to(dev) if c1 else None
    out = ops.group_norm(a, groups, 1e-5, gamma, beta, silu, x2=b)
    multi = ops.group_norm_apply(a, ops.group_norm_stats(a, groups, 1e-5, gamma, beta, x2=b), silu, x2=b)
    diff = (out.float() - multi.float()).abs().max().item()
    assert diff <= 2e-3 * max(1.0, multi.float().abs().max().item()), diff
    pad = ops.group_norm(a, groups, 1e-5, gamma, beta, silu, x2=b, pad=True)
    assert torch.equal(pad[:, 1:-1, 1:-1], out), "padded form's interior == the plain form"
    border = torch.ones(h + 2, w + 2, dtype=torch.bool, device=dev)
    border[1:-1, 1:-1] = False
    assert (pad[:, border] == 0).all()


# GroupNorm with |mean| >> std (the shifted per-block moments keep the variance exact) on the
# plain and the zero-bordered layout, concatenated inputs included; two back-to-back calls give
# bit-identical outputs
@pytest.mark.parametrize("n,h,c0,c1,mean", [(4, 64, 320, 0, 200.0), (16, 32, 640, 0, -50.0), (2, 64, 320, 320, 80.0)])
def test_groupnorm_large_mean(dev, n, h, c0, c1, mean):
    c = c0 + c1
    x0 = gen(n, c0, h, h, seed=75) + mean
    x1 = gen(n, c1, h, h, seed=76) * 2 + mean if c1 else None
    gamma, beta = gen(c, seed=77) * 0.1 + 1, gen(c, seed=78) * 0.1
    a = nhwc(x0).half().to(dev)
    b = nhwc(x1).half().to(dev) if c1 else None
    ref = F.silu(F.group_norm(torch.cat([nchw(a.float().cpu())] + ([nchw(b.float().cpu())] if c1 else []), 1),
                              32, gamma, beta, 1e-5))
    g, bt = gamma.float().to(dev), beta.float().to(dev)
    out = ops.group_norm(a, 32, 1e-5, g, bt, True, x2=b)
    out2 = ops.group_norm(a, 32, 1e-5, g, bt, True, x2=b)
    close(nchw(out), ref, tol_max=5e-3, tol_l2=1e-3)
    assert torch.equal(out, out2)
    pad = ops.group_norm(a, 32, 1e-5, g, bt, True, x2=b, pad=True)
    assert torch.equal(pad[:, 1:-1, 1:-1], out)
    assert (pad[:, 0] == 0).all() and (pad[:, -1] == 0).all() and (pad[:, :, 0] == 0).all() and (pad[:, :, -1] == 0).all()


# VAE widths: the planner's 256x128 (128 channels) and 256x256 (256 / 512 channels)
# variants of the 32x32 tile; torch fp32 on the device is the reference
@pytest.mark.parametrize("n,h,cin,cout", [
    (2, 256, 128, 128),    # 256x128 tile, 3-stage ring
    (2, 128, 256, 512),    # 256x256 tile
    (1, 256, 512, 256),    # 256x256 tile, 18 K steps per 64 channels x 9 taps
])
def test_m32_vae_width_tiles(dev, n, h, cin, cout):
    x = gen(n, cin, h, h, seed=90).to(dev)
    w = gen(cout, cin, 3, 3, seed=91, scale=1 / math.sqrt(9 * cin)).to(dev)
    b = (gen(cout, seed=92) * 0.1).to(dev)
    r = gen(n, cout, h, h, seed=93).to(dev)
    xh, rh = x.half(), r.half()
    ref = F.conv2d(xh.float(), w, b, padding=1) + rh.float()
    wp, kp = ops.pack_conv_weight(w)
    out = ops.conv(nhwc(xh), wp, kp, cout, ksize=3, bias=b.float(), resid=nhwc(rh))
    close(nchw(out), ref)


# LayerNorm: the lanes-per-row kernel at the UNet / HTSAT widths (8 * LPR * CPL
# channels), ragged row counts, a strided input view, and a width that falls back to
# the one-wave-per-row kernel
@pytest.mark.parametrize("m,c,ld", [
    (4099, 320, 320), (1027, 640, 640), (259, 1280, 1280), (333, 96, 96), (97, 768, 768),
    (130, 320, 960),      # column slice of a wider buffer
    (77, 136, 136),       # 17 chunks: generic kernel
])
def test_layernorm_widths(dev, m, c, ld):
    base = gen(m, ld, seed=94) * 2 + 0.7
    gamma, beta = gen(c, seed=95) * 0.1 + 1, gen(c, seed=96) * 0.1
    xd = base.half().to(dev)[:, :c]
    ref = F.layer_norm(xd.float().cpu(), (c,), gamma, beta, 1e-5)
    y = ops.layer_norm(xd, gamma.float().to(dev), beta.float().to(dev), 1e-5)
    close(y, ref, tol_max=5e-3, tol_l2=1e-3)


@pytest.mark.parametrize("rows,cols,scale", [(64, 4096, 8.0), (33, 9216, 4.0), (5, 264, 1.0), (3, 16384, 2.0)])
def test_softmax_rows(dev, rows, cols, scale):
    x = gen(rows, cols, seed=47, scale=scale)
    ref = torch.softmax(x.half().float(), dim=1)
    out = ops.softmax_rows(x.half().to(dev))
    close(out, ref)
    assert ((out.float().sum(1).cpu() - 1).abs() < 1e-2).all()


@pytest.mark.parametrize("b,h,w", [(2, 16, 16), (1, 8, 8)])
def test_vae_attention(dev, b, h, w):
    # AutoencoderKL mid-block attention (GN 32 groups eps 1e-6, one 512-wide head) vs fp32 torch
    from clap2diffusion_amd.vae import VAEAttention
    c = 512
    x = gen(b, h, w, c, seed=48)
    ws = [gen(c, c, seed=50 + i, scale=c ** -0.5) for i in range(4)]
    bs = [gen(c, seed=60 + i, scale=0.1) for i in range(4)]
    gam, bet = 1 + gen(c, seed=70, scale=0.1), gen(c, seed=71, scale=0.1)
    m = VAEAttention(c)
    m.group_norm.load(gam, bet)
    for lin, wt, bi in zip([m.to_q, m.to_k, m.to_v, m.to_out[0]], ws, bs):
        lin.load(wt, bi)
    m.finalize()
    m.to(dev)
    xh = x.half().float()
    xn = F.group_norm(xh.permute(0, 3, 1, 2), 32, gam, bet, 1e-6).permute(0, 2, 3, 1).reshape(b, h * w, c)
    q, k, v = (F.linear(xn, wt, bi) for wt, bi in zip(ws[:3], bs[:3]))
    o = F.scaled_dot_product_attention(q, k, v)
    ref = (F.linear(o, ws[3], bs[3]).view(b, h, w, c) + xh)
    out = m(x.half().to(dev))
    close(out, ref)


@pytest.mark.parametrize("b,l,causal", [(2, 77, True), (3, 77, False), (1, 128, True), (2, 5, True)])
def test_attention_small(dev, b, l, causal):
    h, d = 12, 64
    qkv = gen(b * l, 3 * h * d, seed=80)
    c = h * d
    qh, kh, vh = (qkv[:, i * c:(i + 1) * c].reshape(b, l, h, d).transpose(1, 2) for i in range(3))
    ref = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal).transpose(1, 2).reshape(b * l, c)
    qd = qkv.half().to(dev)
    out = ops.attention_small(qd[:, :c], qd[:, c:2 * c], qd[:, 2 * c:], b, h, l, d, causal=causal)
    close(out, ref)


def test_clip_text_tower(dev):
    # HIP CLIP ViT-L/14 text tower vs transformers' CLIPTextModel in fp32, both loading
    # the seeded CLIPTextModel-keyed state dict (weights.synth_clip_text)
    from clap2diffusion_amd.text_encoder import TextEncoder, tokenize
    from oracle.clip_ref import encode
    ids = tokenize(["", "a beach", "thunder over a dark city street at night"])
    ref = encode(ids, seed=0)
    out = TextEncoder(dev, seed=0)(ids)
    assert out.shape == ref.shape and out.dtype == torch.float16
    close(out, ref, tol_max=3e-2, tol_l2=1e-2)


@pytest.mark.parametrize("cout,cin,k,cin_pad", [(320, 4, 3, 8), (640, 320, 3, None), (1280, 768, 1, None),
                                                 (77, 100, 1, None), (128, 512, 3, None)])
def test_pack_weights_matches_host_packer(dev, cout, cin, k, cin_pad):
    # c2d_pack_weights is bit-identical to the host packer the layers use
    w = gen(cout, cin, k, k, seed=90) if k == 3 else gen(cout, cin, seed=90)
    ref, kp_ref = (ops.pack_conv_weight(w, cin_pad=cin_pad) if k == 3 else ops.pack_linear_weight(w))
    out, kp = ops.pack_weights_device(w.to(dev), cin_pad=cin_pad)
    assert kp == kp_ref and torch.equal(out.cpu(), ref)


# producer-emitted GroupNorm moments (c2d_conv_desc::gn_mom, round 6): the row-ring conv's epilogue
# (one slice) or the split-K combine (splitk_reduce_gn_kernel) writes {mean, M2} per (image, row block,
# group) of the fp16 values it stores; c2d_groupnorm_moments normalises from them.  Against torch fp32
# GroupNorm of the stored conv output and against the statistics pass (c2d_groupnorm) on the same
# tensor; |mean| >> std via a large bias.
@pytest.mark.parametrize("tile,split,n,h,cin,cout,temb,mean,pad,silu", [
    (42, 1, 2, 64, 320, 320, False, 0.0, True, True),     # L0 conv2 (+ residual) -> padded norm (tile 42, 256 rows)
    (42, 1, 2, 64, 320, 320, True, 40.0, False, False),   # + time embedding, |mean| >> std
    (43, 1, 4, 32, 320, 640, True, 0.0, True, True),      # L1 conv1 (tile 43, 128 rows, 20 channels per group)
    (43, 1, 2, 32, 640, 640, False, -25.0, False, True),
    (42, 5, 2, 64, 640, 320, True, 0.0, True, True),      # c2's L0 up conv: row ring, 5 slices -> the combine emits
    (7, 4, 2, 64, 320, 320, False, 30.0, True, True),     # c2's L0 conv: 128 x 320 DMA tile, 4 slices
    (43, 5, 2, 32, 640, 640, True, 0.0, False, True),     # c2's L1 conv: row ring, 5 slices
    (40, 1, 2, 64, 320, 320, False, 20.0, True, True),    # the 256 x 320 ping-pong tile's workgroup epilogue
])
def test_conv_gn_moments(dev, force_plan, tile, split, n, h, cin, cout, temb, mean, pad, silu):
    force_plan(tile, split)
    groups, eps = 32, 1e-5
    x = gen(n, cin, h, h, seed=301)
    w = gen(cout, cin, 3, 3, seed=302, scale=1.0 / math.sqrt(9 * cin))
    b = gen(cout, seed=303) + mean
    r = gen(n, cout, h, h, seed=304)
    te = gen(n, cout, seed=305) if temb else None
    gamma, beta = gen(cout, seed=306).abs() + 0.5, gen(cout, seed=307)
    wp, kp = ops.pack_conv_weight(w)
    xp = F.pad(nhwc(x), (0, 0, 1, 1, 1, 1)).half().to(dev)   # zero-bordered source
    with ops.record_conv_plans() as plans:
        y, mom = ops.conv(xp, wp.to(dev), kp, cout, ksize=3, bias=b.float().to(dev), padded=True,
                          temb=te.half().to(dev) if temb else None, resid=None if temb else nhwc(r).half().to(dev),
                          gn_moments=groups)
    rows = 16 if split > 1 else (256 if tile in (40, 42) else 128)
    assert plans == [(tile, split)] and mom is not None and mom.rows == rows, (plans, mom and mom.rows)
    g, bt = gamma.float().to(dev), beta.float().to(dev)
    got = ops.group_norm(y, groups, eps, g, bt, silu, pad=pad, mom=mom)
    ref_stats = ops.group_norm(y, groups, eps, g, bt, silu, pad=pad)   # the statistics pass on the same tensor
    ref = F.group_norm(nchw(y.float().cpu()), groups, gamma, beta, eps)
    if silu:
        ref = F.silu(ref)
    ref = nhwc(ref)
    if pad:
        assert got.shape == (n, h + 2, h + 2, cout) and got[:, 0].abs().max() == 0 and got[:, :, -1].abs().max() == 0
        got, ref_stats = got[:, 1:-1, 1:-1], ref_stats[:, 1:-1, 1:-1]
    close(got, ref, tol_max=1e-2, tol_l2=2e-3)
    close(got, ref_stats, tol_max=1e-2, tol_l2=2e-3)
    # the emitted moments themselves: per (image, group) mean / variance against fp64 over the stored output
    yg = y.double().cpu().reshape(n, h * h, groups, cout // groups)
    m_ref = yg.mean(dim=(1, 3))
    v_ref = yg.var(dim=(1, 3), unbiased=False)
    mm = mom.mom.double().cpu()   # [n][blocks][groups][2]
    cnt = mom.rows * (cout // groups)
    m_all = mm[..., 0].mean(1)
    m2 = mm[..., 1].sum(1) + cnt * ((mm[..., 0] - m_all[:, None]) ** 2).sum(1)
    v_all = m2 / (cnt * mm.shape[1])
    assert torch.allclose(m_all, m_ref, rtol=1e-5, atol=1e-4 * v_ref.sqrt().max().item())
    assert torch.allclose(v_all, v_ref, rtol=2e-3)


def test_conv_gn_moments_refused_where_not_emitted(dev):
    """A conv whose epilogue cannot emit moments (no residual / time embedding: the per-wave image
    epilogue) returns none; the C entry refuses a descriptor asking for them (C2D_E_SHAPE) rather than
    leaving them unwritten."""
    import ctypes
    from clap2diffusion_amd import torch_ops
    from clap2diffusion_amd._lib import lib
    x = torch.randn(16, 64, 64, 320, device=dev, dtype=torch.float16)
    wp = torch.randn(320, 2880, device=dev, dtype=torch.float16) * 0.02
    y, mom = ops.conv(x, wp, 2880, 320, ksize=3, gn_moments=32)
    assert mom is None
    out = torch.empty_like(x)
    mbuf = torch.empty(16 * 16 * 32 * 2, device=dev)
    d = torch_ops._conv_desc(x, wp, 2880, 320, 3, 1, False, None, None, None, False, None, None, None, False, None, 0,
                             None, None, out, False, 0.0, mbuf, 32)
    assert lib().c2d_conv2d_gn_rows(ctypes.byref(d)) == 0
    assert lib().c2d_conv2d_igemm(ctypes.byref(d), None) == -2
