"""Achievable-bandwidth probe for the bench's access pattern: 8 GiB streamed in place
(read + write) by torch's vectorized elementwise kernel, and an 8 GiB -> 8 GiB copy."""
import time

import torch

n = 1 << 31                                    # floats = 8 GiB
x = torch.rand(n, device="cuda")
y = torch.empty_like(x)
for name, fn in (("inplace_mul", lambda: x.mul_(1.0000001)), ("copy", lambda: y.copy_(x))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 10
    print(f"{name}: {ms:.3f} ms/pass, {2 * n * 4 / ms * 1e-6:.1f} GB/s (read+write)")
