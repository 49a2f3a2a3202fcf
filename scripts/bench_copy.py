"""HBM write/copy baselines at the UNet's level-0 activation size (42 MB fp16)."""
import torch
dev = torch.device("cuda")
x = torch.randn(65536, 320, device=dev).half()
y = torch.empty_like(x)
def t(fn, it=20):
    for _ in range(3): fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); e1.synchronize()
    return e0.elapsed_time(e1) / it * 1e3
us = t(lambda: y.copy_(x)); print(f"copy 42MB: {us:.1f} us  {2*x.numel()*2/us/1e6:.2f} TB/s")
us = t(lambda: y.fill_(1.0)); print(f"fill 42MB: {us:.1f} us  {x.numel()*2/us/1e6:.2f} TB/s")
