#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py into
profiles/pmc_<workload>.json (read by bench.py for roofline.traffic).

The op under test may be several kernels (decode v4: index_kernel +
exec_kernel + the fallback pass); the per-launch traffic is the sum over the
op's kernels of each kernel's average over its dispatches.

    python tools/pmc_summary.py WORKLOAD FETCH.csv WRITE.csv ALGO_BYTES [PIPES_PER_OP]

PIPES_PER_OP (compress only, default 1): encode_pipe_kernel launches per
compress op -- 1 when no message is split (C3: 64 KiB bodies), 2 when the
batch has split messages (the second is the fallback pass).

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
    "decompress": ("fsg::index_kernel", "fsg::index_plan_kernel", "fsg::index_big_kernel",
                   "fsg::exec_kernel", "fsg::decode_pipe_kernel"),
    "compress": ("fsg::encode_plan_kernel", "fsg::encode_pipe_kernel", "fsg::encode_gather_kernel"),
}


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        # "void fsg::index_kernel<false>(...)" -> "fsg::index_kernel"
        name = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("void ", "", 1))
        vals[name].append(float(r["Counter_Value"]))
    return vals


def main():
    workload, fetch_csv, write_csv, algo = sys.argv[1:5]
    pipes_per_op = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    op = "decompress" if workload.endswith("decompress") else "compress"
    names = OP_KERNELS[op]
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    out = {"workload": workload, "kernels": {}}
    fetch_kb = write_kb = 0.0
    for k in set(f) | set(w):
        if not any(k.endswith(n.split("::")[-1]) for n in names):
            continue
        fa = sum(f.get(k, [0])) / max(1, len(f.get(k, [])))
        wa = sum(w.get(k, [0])) / max(1, len(w.get(k, [])))
        # per-dispatch averages: encode_pipe runs pipes_per_op times per compress op
        mult = pipes_per_op if (op == "compress" and k.endswith("encode_pipe_kernel")) else 1
        scale = FETCH_SCALE.get(k.split("::")[-1], 1.0)
        out["kernels"][k] = {"fetch_kb": round(fa, 1), "write_kb": round(wa, 1), "fetch_scale": scale,
                             "dispatches": len(f.get(k, []))}
        fetch_kb += fa * mult * scale
        write_kb += wa * mult
    import bench
    out["kernel_src"] = bench.kernel_source_hash()
    out["fetch_size_kb_per_launch_corrected"] = round(fetch_kb, 1)
    out["write_size_kb_per_launch"] = round(write_kb, 1)
    out["traffic_bytes_per_launch"] = int((fetch_kb + write_kb) * 1024)
    out["algorithmic_bytes_per_launch"] = int(algo)
    out["source"] = f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes ({fetch_csv}, {write_csv})"
    dst = REPO / "profiles" / f"pmc_{workload}.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
