"""H2D DMA rate from pinned host memory: one stream vs two, 7 MB copies (a config B batch)."""
import time

import torch

n = 7 << 20
reps = 64
h = [torch.empty(n, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
d = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(4)]
for x in h:
    x.fill_(1)
for k in range(16):  # first touch of both sides
    d[k % 4].copy_(h[k % 4], non_blocking=True)
streams = [torch.cuda.Stream() for _ in range(4)]
for ns in (1, 2, 4, 1, 2, 4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(reps):
        s = streams[k % ns]
        with torch.cuda.stream(s):
            d[k % 4].copy_(h[k % 4], non_blocking=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"streams {ns}: {reps * n / dt / 1e9:.1f} GB/s")
