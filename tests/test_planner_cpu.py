"""The implicit-GEMM planner (c2d_conv2d_igemm_plan: host code, no GPU needed): the measured
plan table for the SD1.5 UNet shapes at the c2 / c3 / c5 batches (igemm.hip kPlanHints,
profiles/r03_sweep_*.txt) routes those shapes, and a shape the table does not hold falls
through to the rules."""
import ctypes

import pytest


def _plan(cin, cout, n, h, k, ws=True, geglu=False, c1=0):
    import torch  # noqa: F401  (binds the library to torch's HIP runtime first)
    from clap2diffusion_amd import _lib, ops
    L = _lib.lib()
    d = _lib.ConvDesc()
    d.c0, d.c1, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride = cin, c1, n, h, h, h, h, k, 1
    d.cout, d.kpad = cout, ops.kpad_of(k * k * (cin + c1))
    if geglu:
        d.act = 1   # C2D_ACT_GEGLU
    if ws:   # a workspace large enough for any split (the planner only reads the pointer / size)
        d.ws, d.ws_bytes = 16, 1 << 40
    tile, split = ctypes.c_int(-1), ctypes.c_int(-1)
    assert L.c2d_conv2d_igemm_plan(ctypes.byref(d), ctypes.byref(tile), ctypes.byref(split)) == 0
    return tile.value, split.value


@pytest.mark.parametrize("cin,cout,n,h,k,geglu,want", [
    (320, 320, 2, 64, 3, False, (7, 4)),        # c2: L0 resnet conv
    (640, 640, 2, 32, 3, False, (7, 8)),        # c2: L1 resnet conv
    (2560, 1280, 2, 16, 3, False, (41, 16)),    # c2: L2 up-block conv (split 16)
    (1280, 1280, 2, 8, 3, False, (81, 12)),     # c2: L3 resnet conv (two K groups, split 12)
    (1280, 1280, 2, 16, 1, False, (3, 1)),      # c2: L2 projections
    (640, 5120, 2, 32, 1, True, (50, 1)),       # c2: L1 GEGLU (persistent tile)
    (320, 320, 8, 96, 1, False, (7, 1)),        # c5: L0 projections
    (640, 640, 8, 48, 3, False, (41, 1)),       # c5: L1 resnet conv
    (1280, 1280, 16, 16, 1, False, (80, 1)),    # c3: L2 projections (128 x 160, two K groups)
    (1280, 1280, 16, 8, 1, False, (3, 1)),      # c3: mid-block projections
    (256, 128, 8, 512, 1, False, (1, 1)),       # VAE decoder 512^2 shortcut
    (6400, 1280, 16, 16, 1, False, (80, 1)),    # c3: L2 ff.net.2 + proj_out fold (K = 5C)
    (3200, 640, 8, 48, 1, False, (41, 1)),      # c5: L1 fold
    (6400, 1280, 2, 8, 1, False, (3, 12)),      # c2: L3 fold
])
def test_plan_table_routes_unet_shapes(cin, cout, n, h, k, geglu, want):
    assert _plan(cin, cout, n, h, k, geglu=geglu) == want


def test_table_split_needs_workspace_and_other_shapes_use_the_rules():
    # without a workspace a split-K table entry keeps its tile and runs one K slice
    assert _plan(320, 320, 2, 64, 3, ws=False) == (7, 1)
    # c3's level-0 resnet conv is not in the table: the rules' 256 x 320 ping-pong tile
    assert _plan(320, 320, 16, 64, 3) == (40, 1)



def _ws(cin, cout, n, h, k, c1=0):
    import torch  # noqa: F401
    from clap2diffusion_amd import _lib, ops
    d = _lib.ConvDesc()
    d.c0, d.c1, d.n, d.h, d.w, d.oh, d.ow, d.ksize, d.stride = cin, c1, n, h, h, h, h, k, 1
    d.cout, d.kpad = cout, ops.kpad_of(k * k * (cin + c1))
    return _lib.lib().c2d_conv2d_igemm_workspace_size(ctypes.byref(d))


def test_quantisation_tail_reports_the_head_plan():
    """c5's level-0 3x3 convs plan one K slice on 288 tiles of 256 x 320 (one round of 256 CUs +
    32 tiles): c2d_conv2d_igemm runs the first 7 images on that plan and the 8th on its own plan
    (igemm.hip tail_images; the tail's plan here fills the chip without split-K, so the call asks
    for no workspace).  c2d_conv2d_igemm_plan reports the head's plan."""
    assert _plan(320, 320, 8, 96, 3) == (40, 1)
    assert _ws(320, 320, 8, 96, 3) == 0
    assert _plan(320, 320, 1, 96, 3) == (3, 1)           # what the tail image runs
    assert _plan(320, 320, 16, 64, 3) == (40, 1) and _ws(320, 320, 16, 64, 3) == 0   # c3: exact fit


@pytest.mark.parametrize("c0,c1", [(320, 320), (640, 320)])
def test_quantisation_tail_split_k_workspace(c0, c1):
    """The up-block concat convs of c5 (640 / 960 -> 320 at 96^2, 8 images) split the same way, and
    their tail image plans split-K 3 on the 128 x 320 tile: the workspace the call asks for is
    exactly the tail's slabs (3 x 9216 rows x 320 x fp32), not the head's (one slice, none).
    tests/test_kernels_gpu.py::test_conv_quantisation_tail runs these cases on the GPU."""
    assert _plan(c0, 320, 8, 96, 3, c1=c1) == (40, 1)
    assert _plan(c0, 320, 1, 96, 3, c1=c1) == (7, 3)
    assert _ws(c0, 320, 8, 96, 3, c1=c1) == 3 * 9216 * 320 * 4


@pytest.mark.parametrize("n,h,cin,cout,resid,temb,groups,want", [
    (16, 64, 320, 320, True, False, 32, 256),    # c3 L0 conv2 (+ residual) on tile 42: 256-row blocks
    (16, 64, 320, 320, False, True, 32, 256),    # c3 L0 conv1 (+ temb)
    (16, 32, 640, 640, True, False, 32, 128),    # c3 L1 on tile 43: 128-row blocks
    (16, 64, 320, 320, False, False, 32, 0),     # no residual / temb: the per-wave epilogue emits none
    (16, 64, 320, 320, True, False, 30, 0),      # 320 / 30 groups do not tile the 320-column block
    (2, 64, 320, 320, True, False, 32, 16),      # c2 L0: (7, 4) split K -> the combine emits, 16-row blocks
    (2, 64, 640, 320, True, False, 32, 16),      # c2 L0 up conv: the row ring with split K (42, 5)
    (2, 8, 1280, 1280, True, False, 32, 16),     # c2 L3 (81, 12): 8 x 8 = 64 pixels per image, four 16-row blocks
    (2, 8, 1280, 1280, True, False, 128, 16),    # 128 groups of 10 channels tile the block too
])
def test_gn_moment_rows(n, h, cin, cout, resid, temb, groups, want):
    """c2d_conv2d_gn_rows: which convs can emit their output's GroupNorm moments (c2d_conv_desc::gn_mom)
    -- the one-slice row-ring plans with the workgroup-image epilogue -- as ops.gn_moment_rows asks it."""
    from clap2diffusion_amd import ops
    assert ops.gn_moment_rows(n, h, h, cin, cout, 3, 1, True, resid, temb, groups) == want
