"""Pinned host<->device copy bandwidth on this box: one stream vs several
streams in parallel (chunks of one buffer).  Used to size the end-to-end
path's copy pipeline; run twice, with and without HSA_ENABLE_SDMA=0."""
import os
import sys
import time

import torch

N = 2 << 30
h = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h.fill_(1)
d = torch.empty(N, dtype=torch.uint8, device="cuda")
tag = os.environ.get("HSA_ENABLE_SDMA", "default")
for ns in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    for direction in ("h2d", "d2h"):
        best = 1e9
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.perf_counter()
            step = N // ns
            for i, s in enumerate(streams):
                with torch.cuda.stream(s):
                    if direction == "h2d":
                        d[i * step:(i + 1) * step].copy_(h[i * step:(i + 1) * step], non_blocking=True)
                    else:
                        h[i * step:(i + 1) * step].copy_(d[i * step:(i + 1) * step], non_blocking=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        print(f"sdma={tag} streams={ns} {direction} {N / best / 1e9:.1f} GB/s", flush=True)
