"""H2D rate of the bench's end-to-end buffers (pinned host tensor filled from a
device tensor through .cpu(), 2.13 GB) vs a buffer filled on the host."""
import time

import torch

N = 2134156024
src = torch.randint(0, 255, (N,), dtype=torch.uint8, device="cuda")
d = torch.empty_like(src)


def rate(h, what):
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    print(f"{what}: h2d {N / best / 1e9:.1f} GB/s", flush=True)


h1 = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h1.copy_(src.cpu())
rate(h1, "pinned, filled via .cpu()")
h2 = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h2.fill_(3)
rate(h2, "pinned, filled on host")
h3 = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h3.copy_(src, non_blocking=False)
rate(h3, "pinned, filled by D2H")
rate(h1, "first buffer again")
