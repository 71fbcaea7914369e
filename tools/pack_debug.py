#!/usr/bin/env python3
"""Packed execution pass check: decodes a mixed batch on the forked path with
the given exec_pack and reports statuses and mismatching bodies.

    FSG_LIB=... python tools/pack_debug.py --n 20000 --pack 32
"""
import argparse
import collections
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))
import fsg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--pack", type=int, default=32)
    ap.add_argument("--skew", type=int, default=0)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    b = fsg.make_batch(fsg.KIND_MIXED, fsg.mixed_sizes(args.n))
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    n = args.n
    caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
    c_off, c_tot = fsg.slot_offsets(caps)
    codec = fsg.SnappyGPU(0)
    d_c = torch.zeros(c_tot, dtype=torch.uint8, device="cuda")
    d_cl = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
    ws = codec.compress_workspace(n, int(b.lens.max()))
    codec.compress(H(b.data), H(b.offsets), H(b.lens), n, int(b.lens.max()), d_c, H(c_off), d_cl, d_st, workspace=ws)
    torch.cuda.synchronize()
    assert int((d_st != 0).sum()) == 0
    fsg.set_option("decode_fork", 1)
    fsg.set_option("exec_pack", args.pack)
    oo, tot = fsg.slot_offsets(b.lens.astype(np.uint64) + 16)
    oo = oo + (np.arange(n, dtype=np.uint64) * args.skew) % 16
    d_out = torch.full((tot,), 0xA5, dtype=torch.uint8, device="cuda")
    d_ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_st2 = torch.full((n,), -7, dtype=torch.int32, device="cuda")
    dws = codec.decompress_workspace(n, c_tot)
    print("decoding", flush=True)
    codec.decompress(d_c, H(c_off), d_cl, n, d_out, H(oo), H(b.lens), d_ol, d_st2, workspace=dws)
    torch.cuda.synchronize()
    print("decoded", flush=True)
    st = d_st2.cpu().numpy()
    out = d_out.cpu().numpy()
    cl = d_cl.cpu().numpy()
    print("statuses", collections.Counter(st.tolist()).most_common(8))
    bad = []
    for i in range(n):
        o = out[int(oo[i]):int(oo[i]) + int(b.lens[i])].tobytes()
        if st[i] != 0 or o != b.item(i):
            bad.append(i)
    print("bad", len(bad))
    for i in bad[:20]:
        o = out[int(oo[i]):int(oo[i]) + int(b.lens[i])].tobytes()
        ref = b.item(i)
        first = next((k for k in range(len(ref)) if o[k] != ref[k]), -1)
        print(f"  body {i}: len {b.lens[i]} comp {cl[i]} status {st[i]:#x} first diff {first} "
              f"slot {int(oo[i])} got {o[first:first + 8].hex()} ref {ref[first:first + 8].hex()}")
        c = d_c[int(c_off[i]):int(c_off[i]) + int(cl[i])].cpu().numpy().tobytes()
        print("    comp tail", c[-24:].hex())


if __name__ == "__main__":
    main()
