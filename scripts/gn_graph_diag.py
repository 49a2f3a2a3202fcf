"""Diagnostic for the removed single-launch GroupNorm (norm.hip at commit 818994c, C2D_GN_ZERO selected how
its barrier words were zeroed): the words after eager calls and after graph replays (workspace allocated
outside the capture, so it can be read back).  Against the current library c2d_groupnorm runs the
two-launch path, which has no barrier words: the script then only checks replay == eager."""
import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from clap2diffusion_amd import _lib  # noqa: E402

lib = _lib.lib()
dev = torch.device("cuda")
n, h, w, c, groups = 2, 64, 64, 320, 32
x = (torch.randn(n, h, w, c, device=dev) + 0.2).half()
g, b = torch.ones(c, device=dev), torch.zeros(c, device=dev)
wsb = lib.c2d_groupnorm_run_workspace_size(n, c, h * w, groups)
ws = torch.full(((wsb + 15) // 16 * 4,), 7, dtype=torch.int32, device=dev)
out = torch.empty_like(x)
p = lambda t: ctypes.c_void_p(t.data_ptr())


def call(stream):
    rc = lib.c2d_groupnorm(p(x), None, c, 0, n, h * w, groups, 1e-5, p(g), p(b), 1, p(out), p(ws), wsb,
                           ctypes.c_void_p(stream.cuda_stream))
    assert rc == 0, rc


def words(tag):
    torch.cuda.synchronize()
    wv = ws[:8].cpu().tolist()
    print(f"{tag}: timeouts={wv[0]} cnt/gen img0={wv[4]}/{wv[5]} img1={wv[6]}/{wv[7]} nan={torch.isnan(out.float()).any().item()}",
          flush=True)


call(torch.cuda.current_stream())
words("eager")
ref = out.clone()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    call(s)
torch.cuda.current_stream().wait_stream(s)
words("eager side stream")
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    call(torch.cuda.current_stream())
ws.fill_(7)
out.zero_()
torch.cuda.synchronize()
for i in range(3):
    graph.replay()
    words(f"replay {i}")
print("replay equals eager:", torch.equal(out, ref), flush=True)
