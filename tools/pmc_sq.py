#!/usr/bin/env python3
"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (any
counters), one line per (kernel, counter): average per dispatch, plus derived
per-wave figures for the SQ counters.

    python tools/pmc_sq.py gpurun_out/pmc_<wl>/.../sq_counter_collection.csv
"""
import csv
import sys
from collections import defaultdict


def main(path):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k in sorted(vals, key=lambda k: -vals[k].get("SQ_WAVE_CYCLES", 0)):
        n = len(disp[k])
        c = {name: v / n for name, v in vals[k].items()}
        print(f"{k[:60]}  dispatches={n}")
        for name in sorted(c):
            print(f"    {name:22s} {c[name]:16.0f}")
        waves = c.get("SQ_WAVES", 0)
        if waves and "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            parts = [f"per wave: cycles {4 * wc / waves:.0f}"]  # SQ_WAVE_CYCLES counts quad-cycles
            for name in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
                if name in c:
                    parts.append(f"{name[9:]} {c[name] / waves:.0f}")
            for name in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
                if name in c and wc:
                    parts.append(f"{name[3:]} {c[name] / wc:.0%}")
            print("    " + ", ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])
