#!/usr/bin/env python3
"""Diagnostic: per-phase cycle totals of the v4 exec kernel (s_memtime stamps).

Loads the stamps build (make stamps -> libflare_snappy_gpu_stamps.so) in place
of the product library, decodes one C3-shaped batch with the two-pass decoder
and prints the cycles per phase, per group and per message.  Not a benchmark:
the stamps themselves cost cycles.
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

PHASES4 = ["fill", "decode+scan", "pieces+prefetch", "slide+pmap+gather", "roundA", "roundsB",
           "flush", "longlit"]
PHASES5 = ["fill", "decode", "scan+checks+slide+prefetch+zero", "classify+roundA loads", "flush",
           "roundA stores", "roundsB", "longlit"]


def main():
    kind = {"text": fsg.KIND_TEXT, "random": fsg.KIND_RANDOM}[sys.argv[1] if len(sys.argv) > 1 else "text"]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
    codec = fsg.SnappyGPU(0)
    lib = codec.lib
    lib.fsg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    b = fsg.make_batch(kind, np.full(n, size, np.uint32))
    dev = torch.device("cuda", 0)
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
    coff, ctot = fsg.slot_offsets(caps)
    d_raw, d_ro, d_rl = H(b.data), H(b.offsets), H(b.lens)
    d_c = torch.zeros(ctot, dtype=torch.uint8, device=dev)
    d_co, d_cl = H(coff), torch.zeros(n, dtype=torch.int32, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    ws = codec.compress_workspace(n, size)
    codec.compress(d_raw, d_ro, d_rl, n, size, d_c, d_co, d_cl, d_st, workspace=ws)
    d_out = torch.zeros(b.total, dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    dws = codec.decompress_workspace(n, ctot)
    variant = int(os.environ.get("FSG_STAMPS_VARIANT", "5"))
    codec.select_kernels(variant, 0)
    PHASES = PHASES5 if variant == 5 else PHASES4
    buf = (ctypes.c_ulonglong * 24)()
    codec.decompress(d_c, d_co, d_cl, n, d_out, d_ro, d_rl, d_ol, d_st, workspace=dws)
    torch.cuda.synchronize()
    lib.fsg_debug_stamps(buf, 1)
    codec.decompress(d_c, d_co, d_cl, n, d_out, d_ro, d_rl, d_ol, d_st, workspace=dws)
    torch.cuda.synchronize()
    lib.fsg_debug_stamps(buf, 1)
    ok = bool(torch.equal(d_out, d_raw)) and int((d_st != 0).sum()) == 0
    tot = sum(buf[k] for k in range(8))
    groups_est = b.total / 480.0  # ~480 output bytes per text group
    print(f"correct={ok} messages={n} total wave-cycles={tot:.3e} per message={tot / n:.0f}")
    for k, name in enumerate(PHASES):
        print(f"  {name:20s} {buf[k] / tot * 100:5.1f}%  {buf[k] / n:10.0f} cyc/msg  "
              f"{buf[k] / groups_est:8.0f} cyc/group(est)")


if __name__ == "__main__":
    main()
