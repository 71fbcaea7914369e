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
