"""The torch.library layer over the C ABI: every op is registered as
c2d::<name> with a schema, has no CPU kernel (a CPU tensor fails in the dispatcher --
no fallback), and traces under FakeTensorMode (fake implementations) without a GPU."""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from clap2diffusion_amd import ops, torch_ops


@pytest.mark.parametrize("name", torch_ops.OPS)
def test_registered_with_schema(name):
    op = getattr(torch.ops.c2d, name).default
    assert op._schema.name == f"c2d::{name}"
    assert "Tensor(a" in str(op._schema)   # every op mutates a caller-allocated output


def test_cpu_tensor_has_no_kernel():
    x = torch.zeros(4, 8, dtype=torch.float16)
    with pytest.raises((NotImplementedError, RuntimeError)):
        torch.ops.c2d.layernorm(x, torch.ones(8), torch.zeros(8), 1e-5, torch.empty_like(x))


def test_fake_tracing_of_the_unet_ops():
    with FakeTensorMode():
        dev = torch.device("cuda", 0)
        x = torch.empty(16, 64, 64, 320, dtype=torch.float16, device=dev)
        w = torch.empty(320, 2880, dtype=torch.float16, device=dev)
        b = torch.empty(320, device=dev)
        y = ops.conv(x, w, 2880, 320, ksize=3, bias=b, resid=x)
        assert y.shape == x.shape and y.dtype == torch.float16
        up = ops.conv(x, torch.empty(320, 2880, dtype=torch.float16, device=dev), 2880, 320, ksize=3, up=True)
        assert up.shape == (16, 128, 128, 320)
        qkv = torch.empty(16 * 4096, 960, dtype=torch.float16, device=dev)
        o = ops.attention(qkv[:, :320], qkv[:, 320:640], qkv[:, 640:], 16, 8, 4096, 4096, 40)
        assert o.shape == (16 * 4096, 320)
        g = ops.group_norm(x, 32, 1e-5, torch.empty(320, device=dev), torch.empty(320, device=dev), True)
        assert g.shape == x.shape
        lin = ops.conv(qkv, torch.empty(320, 960, dtype=torch.float16, device=dev), 960, 320, ksize=1)
        assert lin.shape == (16 * 4096, 320)
        gg = ops.conv(qkv[:, :320].contiguous(), torch.empty(2560, 320, dtype=torch.float16, device=dev), 320, 2560,
                      ksize=1, act="geglu")
        assert gg.shape == (16 * 4096, 1280)
