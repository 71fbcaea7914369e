#!/bin/bash
# FETCH_SIZE calibration probe + exec phase stamps at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/calib; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- build/fetch_probe > $O/fetch_probe.log 2>&1 || { tail -5 $O/fetch_probe.log; exit 1; }
cat $O/fetch_probe.log | grep -v amdgpu.ids
f=$(find $O/fetch -name "*counter_collection.csv" | head -1); cp $f $O/fetch_counters.csv
python - $O/fetch_counters.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:40], r["Counter_Name"], r["Counter_Value"])
PY
timeout -k 10 200 python tools/stamps.py text 65536 65536 > $O/stamps_c3.txt 2>&1 || { tail -5 $O/stamps_c3.txt; exit 1; }
cat $O/stamps_c3.txt
