#!/usr/bin/env python3
"""Diagnostic: per-phase cycle totals of the LZ4 execution pass
(lz4_decode2.hip, s_memtime stamps).  Loads the stamps build (make stamps ->
libflare_snappy_gpu_stamps.so) in place of the product library, decodes the
C3 bodies through LZ4 with the two-pass decoder and prints the cycles per
phase, per group and per message.  Not a benchmark: the stamps cost cycles.

    python tools/l4stamps.py [n] [size]
"""
import ctypes
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
os.environ["FSG_LIB"] = str(REPO / "flare-cpp_amd" / "lib" / "libflare_snappy_gpu_stamps.so")
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fsg  # noqa: E402

PHASES = ["fill", "ring+decode", "long sequence", "scan+slide+prefetch+zero", "round A", "rounds B"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    codec = fsg.SnappyGPU(0)
    lib = codec.lib
    lib.fsg_debug_l4stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    b = fsg.make_batch(fsg.KIND_TEXT, np.full(n, size, np.uint32))
    dev = torch.device("cuda", 0)
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    caps = np.array([lib.fsg_lz4_max_compressed_length(int(x)) for x in b.lens], np.uint64)
    coff, ctot = fsg.slot_offsets(caps)
    d_raw, d_ro, d_rl = H(b.data), H(b.offsets), H(b.lens)
    d_c = torch.zeros(ctot, dtype=torch.uint8, device=dev)
    d_co, d_cl = H(coff), torch.zeros(n, dtype=torch.int32, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    codec.lz4_compress(d_raw, d_ro, d_rl, n, d_c, d_co, d_cl, d_st, codec.lz4_compress_workspace(n))
    d_out = torch.zeros(b.total, dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    dws = codec.lz4_decompress_workspace(n, int(ctot))
    buf = (ctypes.c_ulonglong * 8)()
    for _ in range(2):
        lib.fsg_debug_l4stamps(buf, 1)
        codec.lz4_decompress(d_c, d_co, d_cl, n, d_out, d_ro, d_rl, d_ol, d_st, workspace=dws)
        torch.cuda.synchronize()
    lib.fsg_debug_l4stamps(buf, 1)
    ok = bool(torch.equal(d_out, d_raw)) and int((d_st != 0).sum()) == 0
    tot = sum(buf[k] for k in range(6))
    groups, rounds = buf[6], buf[7]
    print(f"correct={ok} messages={n} wave-cycles={tot:.3e} per message={tot / n:.0f} "
          f"groups/msg={groups / n:.1f} roundsB/group={rounds / max(1, groups):.2f}")
    for k, name in enumerate(PHASES):
        print(f"  {name:26s} {buf[k] / tot * 100:5.1f}%  {buf[k] / n:10.0f} cyc/msg  "
              f"{buf[k] / max(1, groups):8.0f} cyc/group")


if __name__ == "__main__":
    main()
