#!/usr/bin/env python3
"""Kernel timeline of the last decode step in a rocprofv3 kernel_trace.csv:
start/end (us, relative to the step's first kernel) and queue of each kernel.

    python tools/timeline.py .../tr_kernel_trace.csv
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].split("(")[0].replace("void ", "")
rows.sort(key=lambda r: r["s"])
# steps start at the fill before an index/plan kernel: take the last index_plan or index_kernel launch group
starts = [i for i, r in enumerate(rows) if "index_plan_kernel" in r["k"] or "index_kernel<false>" in r["k"]]
i0 = starts[-1] if starts else 0
# include the fills just before
while i0 > 0 and "fill" in rows[i0 - 1]["k"].lower() and rows[i0]["s"] - rows[i0 - 1]["e"] < 50000:
    i0 -= 1
t0 = rows[i0]["s"]
end = max(r["e"] for r in rows[i0:] if "fsg::" in r["k"] or "rocclr" in r["k"])
for r in rows[i0:]:
    if r["s"] > end:
        break
    print(f"{(r['s'] - t0) / 1e3:9.1f} {(r['e'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f} us  q{r.get('Queue_Id', r.get('Stream_Id', '?'))}  {r['k'][:60]}")
print(f"step span {(end - t0) / 1e3:.1f} us")
