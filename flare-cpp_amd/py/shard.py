"""Message sharding across the GPUs of one node.

Snappy messages are independent, so the path shards with no data-path
collective: each rank owns a contiguous range of message indices.  Two modes:

* weak   -- every rank owns a full batch of its own messages
            ([rank*n, (rank+1)*n)); per-GPU work fixed as N grows.
* strong -- one global batch split into contiguous ranges balanced by
            cumulative BYTES (prefix sum of sizes cut at the r/N quantiles),
            not by count: CM's power-law sizes put ~1/3 of the bytes in 0.4%
            of the bodies.

The only collectives are the measurement ones (RCCL over xGMI when the
backend is "nccl"): MAX of per-rank times and SUM of byte / error counters.
"""
from __future__ import annotations

import numpy as np


def weak_range(n_per_rank: int, rank: int) -> tuple[int, int]:
    return rank * n_per_rank, (rank + 1) * n_per_rank


def byte_balanced_ranges(sizes, world: int) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) index ranges whose byte totals are as even as possible."""
    sizes = np.asarray(sizes, dtype=np.uint64)
    n = len(sizes)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(0, world - 1)
    csum = np.cumsum(sizes, dtype=np.uint64)
    total = int(csum[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        # first index whose prefix (inclusive) reaches the target
        k = int(np.searchsorted(csum, np.uint64(target), side="left")) + 1
        k = min(max(k, cuts[-1]), n)
        cuts.append(k)
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def reduce_measurements(dist, device, t_step: float, t_kernel: float, raw_bytes: int, comp_bytes: int,
                        errors: int, bad: int):
    """MAX over ranks of the times, SUM of the counters (the bench's only collectives)."""
    import torch
    t = torch.tensor([t_step, t_kernel], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([raw_bytes, comp_bytes, errors, bad], dtype=torch.int64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t[0]), float(t[1]), [int(x) for x in s.tolist()]
