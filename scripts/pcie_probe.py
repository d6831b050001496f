"""PCIe DMA ceiling on this box: pinned host <-> HBM copy rates, one direction and both at once."""
import time

import torch

n = 1 << 30
h_src = torch.empty(n, dtype=torch.uint8).pin_memory()
h_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
for _ in range(2):
    d_a.copy_(h_src, non_blocking=True)
    h_dst.copy_(d_b, non_blocking=True)
torch.cuda.synchronize()


def timed(fn, reps=5):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


h2d = timed(lambda: d_a.copy_(h_src, non_blocking=True))
d2h = timed(lambda: h_dst.copy_(d_b, non_blocking=True))


def both():
    with torch.cuda.stream(s1):
        d_a.copy_(h_src, non_blocking=True)
    with torch.cuda.stream(s2):
        h_dst.copy_(d_b, non_blocking=True)


bt = timed(both)
print(f"H2D {n / h2d / 1e9:.1f} GB/s  D2H {n / d2h / 1e9:.1f} GB/s  both at once {2 * n / bt / 1e9:.1f} GB/s total")
