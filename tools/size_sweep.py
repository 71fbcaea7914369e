"""Diagnostic: Snappy two-pass decode of uniform text batches of the same
total size (1 GiB) in bodies of different sizes, to expose the per-message
cost of the execution pass.  Prints ms per batch and GiB/s per body size.

    python tools/size_sweep.py [--total-mib 1024] [--sizes 1024,4096,16384,65536]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))
import fsg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-mib", type=int, default=1024)
    ap.add_argument("--sizes", default="1024,4096,16384,65536")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    codec = fsg.SnappyGPU(0)
    H = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    s = torch.cuda.current_stream()
    res = []
    for size in map(int, a.sizes.split(",")):
        n = (a.total_mib << 20) // size
        b = fsg.make_batch(fsg.KIND_TEXT, np.full(n, size, np.uint32))
        d_raw, d_ro, d_rl = H(b.data), H(b.offsets), H(b.lens)
        caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
        coff, ctot = fsg.slot_offsets(caps)
        d_c, d_co = torch.zeros(ctot, dtype=torch.uint8, device=dev), H(coff)
        d_cl = torch.zeros(n, dtype=torch.int32, device=dev)
        d_st = torch.zeros(n, dtype=torch.int32, device=dev)
        ws = codec.compress_workspace(n, size)
        codec.compress(d_raw, d_ro, d_rl, n, size, d_c, d_co, d_cl, d_st, workspace=ws)
        torch.cuda.synchronize()
        del ws
        d_out = torch.zeros(b.total, dtype=torch.uint8, device=dev)
        d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
        dws = codec.decompress_workspace(n, int(ctot))

        def dec():
            codec.decompress(d_c, d_co, d_cl, n, d_out, d_ro, d_rl, d_ol, d_st, stream=s, workspace=dws)

        dec()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.steps):
            dec()
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        ok = int((d_st != 0).sum().item()) == 0 and bool(torch.equal(d_out, d_raw))
        res.append({"size": size, "n": n, "ms": round(ms, 3), "gib_s": round(b.total / (ms / 1e3) / (1 << 30), 1),
                    "us_per_1k_msgs": round(ms * 1e3 / n * 1000, 2), "ok": ok})
        print(json.dumps(res[-1]), flush=True)
        del d_raw, d_c, d_out, dws


if __name__ == "__main__":
    main()
