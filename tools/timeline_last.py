#!/usr/bin/env python3
"""Timeline of the last decode step in a rocprofv3 kernel_trace.csv: every
fsg:: kernel from the last index_plan_kernel (or index_kernel) on, with its
queue, start, end and duration in us relative to the step's first kernel.

    python tools/timeline_last.py gpurun_out/.../kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = [r for r in csv.DictReader(open(path)) if "fsg::" in r["Kernel_Name"] and "encode" not in r["Kernel_Name"]]
    starts = [k for k, r in enumerate(rows) if "index_plan" in r["Kernel_Name"]] or \
             [k for k, r in enumerate(rows) if "index_kernel" in r["Kernel_Name"]]
    sel = rows[starts[-1]:]
    t0 = min(int(r["Start_Timestamp"]) for r in sel)
    print(f"{'kernel':44s} {'queue':>5} {'start':>9} {'end':>9} {'us':>9}")
    for r in sel:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        print(f"{name[:44]:44s} {r.get('Queue_Id', '?'):>5} {s:9.1f} {e:9.1f} {e - s:9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
