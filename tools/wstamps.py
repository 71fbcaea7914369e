#!/usr/bin/env python3
"""Diagnostic: per-phase cycle totals of the wave encoder (s_memtime stamps,
stamps build: make stamps).  Encodes one C3-shaped batch with every message
on the wave encoder and prints the cycles per phase, per block and per
fragment.  Not a benchmark: the stamps cost cycles."""
import ctypes
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
STAMPS = not os.environ.get("FSG_NOSTAMPS")  # FSG_NOSTAMPS=1: the default library, timing only (for --pmc runs)
if STAMPS:
    os.environ["FSG_LIB"] = str(REPO / "flare-cpp_amd" / "lib" / "libflare_snappy_gpu_stamps.so")
os.environ["FSG_ENCODE_WAVE_MIN"] = os.environ.get("FSG_ENCODE_WAVE_MIN", "1")
os.environ["FSG_ENCODE_WAVE_ALL_MB"] = os.environ.get("FSG_ENCODE_WAVE_ALL_MB", "100000")  # every unit on the wave encoder
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fsg  # noqa: E402

PHASES = ["block input", "slots+cand+spec", "pred rounds+permutes", "search", "emit", "commit", "frag setup/tail",
          "match extension"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    codec = fsg.SnappyGPU(0)
    lib = codec.lib
    if STAMPS:
        lib.fsg_debug_wstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    kind = sys.argv[3] if len(sys.argv) > 3 else "text"  # text | proto (SnappyMessageProto, C5's bodies)
    b = fsg.make_batch(fsg.KIND_PROTO if kind == "proto" else fsg.KIND_TEXT, np.full(n, size, np.uint32))
    size = int(b.lens.max())
    dev = torch.device("cuda", 0)
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
    coff, ctot = fsg.slot_offsets(caps)
    d_raw, d_ro, d_rl = H(b.data), H(b.offsets), H(b.lens)
    d_c = torch.zeros(ctot, dtype=torch.uint8, device=dev)
    d_co, d_cl = H(coff), torch.zeros(n, dtype=torch.int32, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    ws = codec.compress_workspace(n, size)
    buf = (ctypes.c_ulonglong * 16)()
    for _ in range(2):
        if STAMPS:
            lib.fsg_debug_wstamps(buf, 1)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        codec.compress(d_raw, d_ro, d_rl, n, size, d_c, d_co, d_cl, d_st, workspace=ws)
        ev1.record()
        torch.cuda.synchronize()
    if not STAMPS:
        print(f"messages={n} size={size} time={ev0.elapsed_time(ev1):.2f} ms")
        return
    lib.fsg_debug_wstamps(buf, 1)
    tot = sum(buf[k] for k in range(8)) + buf[12] + buf[13]
    blocks = max(1, buf[8])
    print(f"messages={n} size={size} time={ev0.elapsed_time(ev1):.2f} ms total wave-cycles={tot:.3e} "
          f"per fragment={tot / n:.0f} per block={tot / blocks:.0f}")
    print(f"  blocks={buf[8]} events/block={buf[9] / blocks:.2f} scans/block={buf[10] / blocks:.3f} "
          f"scan steps/block={buf[11] / blocks:.2f}")
    for k, name in list(enumerate(PHASES)) + [(12, "fast precompute"), (13, "fast walk")]:
        print(f"  {name:24s} {100.0 * buf[k] / max(tot, 1):5.1f}%  {buf[k] / blocks:8.0f} cyc/block")


if __name__ == "__main__":
    main()
