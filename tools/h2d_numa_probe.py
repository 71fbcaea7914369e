"""Pinned H2D / D2H rate of a 2.13 GB buffer allocated by a process bound to
one NUMA node's CPUs (argument: node index), to test whether the bench's
24 GB/s H2D is a remote-node pinned buffer.  Binding happens before torch
touches the GPU.  usage: python tools/h2d_numa_probe.py NODE"""
import os
import sys
import time
from pathlib import Path


def node_cpus(n: int) -> set[int]:
    out = set()
    for part in Path(f"/sys/devices/system/node/node{n}/cpulist").read_text().strip().split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


node = int(sys.argv[1])
os.sched_setaffinity(0, node_cpus(node) & os.sched_getaffinity(0) or node_cpus(node))

import torch  # noqa: E402

N = 2134156024
d = torch.empty(N, dtype=torch.uint8, device="cuda")
h = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h.fill_(3)
res = {}
for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    res[name] = round(N / best / 1e9, 1)
gpu_node = None
try:
    bdf = torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0), "pci_bus_id") else None
except Exception:
    bdf = None
print({"cpu_node": node, "gpu_pci": bdf, **res}, flush=True)
