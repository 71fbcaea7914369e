#!/usr/bin/env python3
"""Diagnostic: per-phase cycle totals of the packed execution pass
(exec5_packed, stamps build: make stamps) on the CM batch, forked path.
Not a benchmark: the stamps cost cycles."""
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

PH = ["fill", "decode", "positions+checks+slide", "roundA issue+prefetch+zero", "flush", "roundA stores",
      "roundsB", "longlit", "setup+singles"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    pack = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    codec = fsg.SnappyGPU(0)
    lib = codec.lib
    lib.fsg_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    b = fsg.make_batch(fsg.KIND_MIXED, fsg.mixed_sizes(n))
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
    coff, ctot = fsg.slot_offsets(caps)
    d_c = torch.zeros(ctot, dtype=torch.uint8, device="cuda")
    d_cl = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
    ws = codec.compress_workspace(n, int(b.lens.max()))
    d_raw = H(b.data)
    codec.compress(d_raw, H(b.offsets), H(b.lens), n, int(b.lens.max()), d_c, H(coff), d_cl, d_st, workspace=ws)
    fsg.set_option("decode_fork", 1, lib)
    fsg.set_option("exec_pack", pack, lib)
    d_out = torch.zeros(b.total, dtype=torch.uint8, device="cuda")
    d_ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    dws = codec.decompress_workspace(n, ctot)
    buf = (ctypes.c_ulonglong * 24)()
    for _ in range(2):
        lib.fsg_debug_stamps(buf, 1)
        codec.decompress(d_c, H(coff), d_cl, n, d_out, H(b.offsets), H(b.lens), d_ol, d_st, workspace=dws)
        torch.cuda.synchronize()
    lib.fsg_debug_stamps(buf, 1)
    ok = bool(torch.equal(d_out, d_raw)) and int((d_st != 0).sum()) == 0
    tot = sum(buf[8 + k] for k in range(9))
    groups, llits, batches, singles = buf[17], buf[18], buf[19], buf[21]
    print(f"ok={ok} pack={pack} batches {batches} groups {groups} long literals {llits} singles {singles}")
    for k, name in enumerate(PH):
        v = buf[8 + k]
        print(f"  {name:30s} {v / max(tot, 1) * 100:5.1f}%  {v / max(groups, 1):8.0f} cycles per group")
    print(f"  total wave-cycles {tot:.3e}; per batch {tot / max(batches, 1):.0f}")
    tot5 = sum(buf[k] for k in range(8))
    print(f"  exec5_message waves (other parts) total {tot5:.3e}")


if __name__ == "__main__":
    main()
