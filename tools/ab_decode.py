#!/usr/bin/env python3
"""A/B of decoder builds in ONE process on one box: the batch is generated and
compressed once, then every library in --libs decodes it in interleaved
rounds (warmup + timed steps each, HIP events on the stream), with the
round trip checked (torch.equal against the raw batch, zero statuses) after
every library's turn.  A library given as path@opt=value,... runs with those
fsg_set_option values.

    python tools/ab_decode.py --workload c3 --libs build/ab/lib_base.so build/ab/lib_new.so
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

WL = {"c3": (fsg.KIND_TEXT, 65536, 65536), "c2": (fsg.KIND_RANDOM, 65536, 4096),
      "cm": (fsg.KIND_MIXED, 1 << 20, None), "c3h": (fsg.KIND_TEXT, 16384, 65536)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=sorted(WL))
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
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
    base = fsg.SnappyGPU(0)
    ws = base.compress_workspace(n, int(b.lens.max()))
    base.compress(d_raw, d_off, d_len, n, int(b.lens.max()), d_c, d_coff, d_cl, d_st, workspace=ws)
    torch.cuda.synchronize()
    del ws
    assert int((d_st != 0).sum()) == 0
    comp_total = int(d_cl.sum().item())
    d_out = torch.full((b.total,), 0xA5, dtype=torch.uint8, device="cuda")
    d_ol = torch.zeros(n, dtype=torch.int32, device="cuda")
    dws = base.decompress_workspace(n, c_tot)
    stream = torch.cuda.current_stream()
    print(f"# {args.workload}: {n} bodies, {b.total} -> {comp_total} bytes, setup {time.time() - t0:.1f} s",
          flush=True)
    runs = []
    for spec in args.libs:
        path, _, opts = spec.partition("@")
        kv = dict(x.split("=") for x in opts.split(",")) if opts else {}
        runs.append((spec, fsg.SnappyGPU(0, Path(path)), {k: int(v) for k, v in kv.items()}))
    res = {spec: [] for spec, _, _ in runs}
    # specs sharing one library path share its option table: every turn
    # starts from the values found at load time, then applies its own
    touched = sorted({k for _, _, kv in runs for k in kv})
    def _known(lib, k):
        try:
            return fsg.get_option(k, lib)
        except KeyError:  # an older library without this option
            return None
    initial = {id(c.lib): {k: v for k in touched if (v := _known(c.lib, k)) is not None} for _, c, _ in runs}
    for r in range(args.rounds):
        for spec, codec, kv in runs:
            for k, v in {**initial[id(codec.lib)], **kv}.items():
                fsg.set_option(k, v, codec.lib)
            step = lambda: codec.decompress(d_c, d_coff, d_cl, n, d_out, d_off, d_len, d_ol, d_st,  # noqa: E731
                                            stream=stream, workspace=dws)
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
            ok = bool(torch.equal(d_out, d_raw)) and int((d_st != 0).sum()) == 0
            d_out.fill_(0xA5)
            res[spec].append(ms)
            print(f"{r} {spec} {ms:.4f} ms ok={ok}", flush=True)
            if not ok:
                print("ROUNDTRIP FAILED", flush=True)
                sys.exit(1)
    summ = {spec: {"min": min(v), "mean": sum(v) / len(v), "all": v} for spec, v in res.items()}
    print(json.dumps({"workload": args.workload, "results": summ}))


if __name__ == "__main__":
    main()
