"""Diagnostic (GPU): decode the randomized parity batch with the two-lane
index walk off and on; print the messages whose status or bytes differ."""
import sys
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parents[1]
for p in (REPO / "flare-cpp_amd" / "py", REPO / "oracle", REPO / "tests"):
    sys.path.insert(0, str(p))
import fsg
from bind import Oracle
from gpu_harness import GpuCodec
import torch
torch.cuda.set_device(0)
o = Oracle()
g = GpuCodec()
rng = np.random.default_rng(3)
items = []
for t in range(400):
    n = int(rng.choice([rng.integers(0, 100), rng.integers(0, 5000), rng.integers(0, 140000)]))
    alpha = int(rng.choice([2, 3, 8, 40, 256]))
    items.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
comps = [o.compress(x) for x in items]
res = {}
for sp in (0, 1):
    fsg.set_option("split_index", sp)
    outs, ol, st = g.decompress(comps, [len(x) for x in items])
    res[sp] = (outs, st)
fsg.set_option("split_index", 1)
for i, (x, c) in enumerate(zip(items, comps)):
    a, b = res[0][1][i], res[1][1][i]
    ok0 = res[0][0][i] == x
    ok1 = res[1][0][i] == x
    if a != b or ok0 != ok1:
        out = res[1][0][i]
        first = next((k for k in range(min(len(out), len(x))) if out[k] != x[k]), None)
        print(f"msg {i}: in {len(x)} comp {len(c)} st0 {a} st1 {b} ok0 {ok0} ok1 {ok1} first_diff {first} head {c[:6].hex()}")
np.save("gpurun_out/debug_split_comps_idx.npy", np.array([len(c) for c in comps]))
print("done")
