#!/usr/bin/env python3
"""A/B of encoder builds in ONE process on one box: the batch is generated
once, then every library in --libs compresses it in interleaved rounds
(warmup + timed steps each, HIP events on the stream).  After every turn
every body's compressed bytes (length and FNV-1a digest) must equal the
first library's and every status be OK; the first library's output is
decoded once and checked against the raw batch.  A library given as
path@opt=value,... runs with those fsg_set_option values.

    python tools/ab_encode.py --workload c5 --libs build/ab/lib_base.so build/ab/lib_new.so
    (workloads: c3, c5; c3w / c5w: every long unit on the wave encoder)
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))
import fsg  # noqa: E402

WL = {"c3": (fsg.KIND_TEXT, 65536, 65536), "c5": (fsg.KIND_PROTO, 262144, None),
      "c3w": (fsg.KIND_TEXT, 65536, 65536), "c5w": (fsg.KIND_PROTO, 262144, None),
      "c3s": (fsg.KIND_TEXT, 8192, 65536),
      "s4k": (fsg.KIND_TEXT, 131072, 4096), "s8k": (fsg.KIND_TEXT, 65536, 8192),
      "s2k": (fsg.KIND_TEXT, 131072, 2048), "c2r": (fsg.KIND_RANDOM, 65536, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c5", choices=sorted(WL))
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    kind, n, size = WL[args.workload]
    sizes = np.full(n, size, np.uint32) if size else fsg.mixed_sizes(n)
    t0 = time.time()
    b = fsg.make_batch(kind, sizes)
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    d_raw, d_off, d_len = H(b.data), H(b.offsets), H(b.lens)
    caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
    c_off, c_tot = fsg.slot_offsets(caps)
    d_c = torch.zeros(c_tot, dtype=torch.uint8, device="cuda")
    d_coff = H(c_off)
    d_cl = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_st = torch.zeros(n, dtype=torch.int32, device="cuda")
    max_len = int(b.lens.max())
    stream = torch.cuda.current_stream()
    print(f"# {args.workload}: {n} bodies, {b.total} bytes, setup {time.time() - t0:.1f} s", flush=True)
    runs = []
    for spec in args.libs:
        path, _, opts = spec.partition("@")
        kv = dict(x.split("=") for x in opts.split(",")) if opts else {}
        kv = {k: int(v) for k, v in kv.items()}
        if args.workload.endswith("w"):
            kv.setdefault("encode_wave_all_mb", 1 << 20)
            kv.setdefault("encode_wave_min", 4096)
        codec = fsg.SnappyGPU(0, Path(path))
        runs.append((spec, codec, kv, codec.compress_workspace(n, max_len)))
    res = {spec: [] for spec, _, _, _ in runs}
    # specs sharing one library path share its option table: every turn
    # starts from the values found at load time, then applies its own
    touched = sorted({k for _, _, kv, _ in runs for k in kv})
    def _known(lib, k):
        try:
            return fsg.get_option(k, lib)
        except KeyError:  # an older library without this option
            return None
    initial = {id(c.lib): {k: v for k in touched if (v := _known(c.lib, k)) is not None} for _, c, _, _ in runs}
    ref_lens = None
    for r in range(args.rounds):
        for spec, codec, kv, ws in runs:
            for k, v in {**initial[id(codec.lib)], **kv}.items():
                fsg.set_option(k, v, codec.lib)
            step = lambda: codec.compress(d_raw, d_off, d_len, n, max_len, d_c, d_coff, d_cl, d_st,  # noqa: E731
                                          stream=stream, workspace=ws)
            for _ in range(args.warmup):
                step()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(args.steps):
                step()
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            # one more pass for the byte comparison: every body's compressed
            # bytes (length + FNV-1a of [offset, offset + length)) against the
            # first library's -- bytes past a body's length are scratch (the
            # lane encoder's 16-byte spill) and are not compared
            step()
            torch.cuda.synchronize()
            ok = int((d_st != 0).sum()) == 0
            lens = d_cl.cpu().numpy().astype(np.uint32)
            dig = fsg.digests(d_c.cpu().numpy(), c_off, lens)
            if ref_lens is None:
                ref_lens, ref_dig = lens, dig
                d_out = torch.full((b.total,), 0xA5, dtype=torch.uint8, device="cuda")
                d_ol = torch.zeros(n, dtype=torch.int32, device="cuda")
                dws = codec.decompress_workspace(n, c_tot)
                codec.decompress(d_c, d_coff, d_cl, n, d_out, d_off, d_len, d_ol, d_st, workspace=dws)
                torch.cuda.synchronize()
                ok = ok and bool(torch.equal(d_out, d_raw)) and int((d_st != 0).sum()) == 0
                del d_out, dws
                print(f"# compressed {int(lens.sum())} bytes; reference output decodes: {ok}", flush=True)
            else:
                bad = np.nonzero((lens != ref_lens) | (dig != ref_dig))[0]
                if len(bad):
                    print(f"# {len(bad)} bodies differ, first {bad[:8].tolist()}", flush=True)
                ok = ok and len(bad) == 0
            res[spec].append(ms)
            print(f"{r} {spec} {ms:.3f} ms ok={ok}", flush=True)
            if not ok:
                print("MISMATCH", flush=True)
                sys.exit(1)
    summ = {spec: {"min": min(v), "mean": sum(v) / len(v), "all": v} for spec, v in res.items()}
    print(json.dumps({"workload": args.workload, "results": summ}))


if __name__ == "__main__":
    main()
