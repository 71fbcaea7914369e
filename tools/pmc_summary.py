#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into
profiles/pmc_<workload>.json (read by bench.py for roofline.traffic).

The op under test may be several kernels (decode v4: index_kernel +
exec_kernel + the fallback pass); the per-launch traffic is the sum over the
op's kernels of each kernel's average over its dispatches.

    python tools/pmc_summary.py WORKLOAD FETCH.csv WRITE.csv ALGO_BYTES

Per op = every dispatch of the op's kernels summed, over the number of ops
the run executed (the dispatches of a kernel each op launches once).

FETCH_SIZE is corrected per kernel by its access pattern (MI355X_MICROARCH.md:
FETCH_SIZE counts half the bytes of wide coalesced 16-B-per-lane reads):
x2 for exec_kernel and index_kernel: on C3 the index pass reads the 2.13 GB
input once and FETCH_SIZE reports 1.06 GB; on C2 exec reads the 0.27 GB input
once and FETCH_SIZE reports 0.16 GB (x2 = 0.33 GB: unaligned 16-B-per-lane
copies touch one extra line per 1 KiB).  The single-pass fallback pass (~0
bytes) keeps x1.  WRITE_SIZE is exact (C2: 262,144 KB = the output).
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

FETCH_SCALE = {"exec_kernel": 2.0, "index_kernel": 2.0, "index_big_kernel": 2.0}
# Where each scale comes from (round 6, tools/probes/fetch_probe.hip,
# profiles/r6/fetch/): FETCH_SIZE counts L2 misses only (16-B sc1 loads over
# an L2-resident 1 MiB: 0.25 B per load) and tallies every missed 128-B line
# at 64 B, for the exec pass's far-load pattern as for streaming: 16-B sc1
# loads at random byte offsets report 68.5 B per load from a 96 MiB
# Infinity-Cache-resident buffer and 71.4 B per load from 2 GiB (64 B per
# line touched, 7-12% of the loads spanning two lines); at x2 the 2 GiB
# kernel moved 5.55 TB/s and random whole-line loads 5.2-5.3 TB/s, beside
# 4.84 TB/s for the calibrated x2 of a coalesced stream -- at x1 a kernel
# with a million threads in flight would reach half the HBM rate a stream
# does.  So the exec pass's far loads take x2 like its input reads.
FETCH_SCALE_SOURCE = {
    "exec_kernel": "profiles/r6/fetch/fp_FETCH_SIZE.csv: far_rand<1>/<2> (16-B sc1 loads at random byte offsets, "
                   "the far-load pattern) 68.5/71.4 B per load = 64 B per 128-B line; x2 as the coalesced "
                   "stream16 (0.5 GiB reported for 1 GiB read)",
    "index_kernel": "profiles/r6/fetch/fp_FETCH_SIZE.csv: stream16 (1 GiB coalesced 16-B reads -> 0.5 GiB reported)",
    "index_big_kernel": "profiles/r6/fetch/fp_FETCH_SIZE.csv: stream16 (as index_kernel)",
}

OP_KERNELS = {
    "decompress": ("index_kernel", "index_plan_kernel", "walk_offsets_kernel", "walk_scatter_kernel",
                   "index_big_kernel", "chunk_list_kernel", "chunk_spec_kernel", "chunk_fixup_kernel",
                   "chunk_check_kernel", "chunk_final_kernel", "exec_kernel", "fallback_kernel",
                   "decode_pipe_kernel"),
    "compress": ("encode_plan_kernel", "encode_pipe_kernel", "encode_wave_kernel", "encode_gather_kernel"),
}
# a kernel every op launches exactly once: its dispatch count is the number of
# ops the profiled run executed (the bench's untimed first call included)
ANCHOR = {"decompress": "fallback_kernel", "compress": "encode_plan_kernel"}


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        # "void fsg::index_kernel<false>(...)" -> "index_kernel"
        name = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("void ", "", 1)).split("::")[-1]
        vals[name].append(float(r["Counter_Value"]))
    return vals


def main():
    workload, fetch_csv, write_csv, algo = sys.argv[1:5]
    op = "decompress" if workload.endswith("decompress") else "compress"
    names = OP_KERNELS[op]
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    n_ops_f = len(f.get(ANCHOR[op], [])) or 1
    n_ops_w = len(w.get(ANCHOR[op], [])) or 1
    out = {"workload": workload, "ops_profiled": n_ops_f, "kernels": {}}
    fetch_kb = write_kb = 0.0
    for k in sorted(set(f) | set(w)):
        if k not in names:
            continue
        # per op: the kernel's dispatches summed (a kernel may run several
        # times per op: the forked decode's three execution launches)
        fa = sum(f.get(k, [])) / n_ops_f
        wa = sum(w.get(k, [])) / n_ops_w
        scale = FETCH_SCALE.get(k, 1.0)
        out["kernels"][k] = {"fetch_kb_per_op": round(fa, 1), "write_kb_per_op": round(wa, 1),
                             "fetch_scale": scale, "dispatches": len(f.get(k, []))}
        if k in FETCH_SCALE_SOURCE:
            out["kernels"][k]["fetch_scale_source"] = FETCH_SCALE_SOURCE[k]
        fetch_kb += fa * scale
        write_kb += wa
    import bench
    out["kernel_src"] = bench.kernel_source_hash()
    out["fetch_size_kb_per_launch_corrected"] = round(fetch_kb, 1)
    out["write_size_kb_per_launch"] = round(write_kb, 1)
    out["traffic_bytes_per_launch"] = int((fetch_kb + write_kb) * 1024)
    out["algorithmic_bytes_per_launch"] = int(algo)
    out["traffic_over_algorithmic"] = round((fetch_kb + write_kb) * 1024 / max(1, int(algo)), 3)
    out["source"] = f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes ({fetch_csv}, {write_csv})"
    dst = REPO / "profiles" / f"pmc_{workload}.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
