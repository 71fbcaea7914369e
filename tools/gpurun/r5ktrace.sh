#!/bin/bash
# Kernel trace + stats of one decode step of $WL through tools/ab_decode.py
# (library spec $LIB, e.g. flare-cpp_amd/lib/libflare_snappy_gpu.so@tiny_pass=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5ktrace}
mkdir -p $O
i=0
for L in $LIBS; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$i -o run -- \
    python tools/ab_decode.py --workload ${WL:-cm} --rounds 1 --steps 2 --warmup 1 --libs $L > $O/t$i.log 2>&1 \
    || { tail -20 $O/t$i.log; exit 1; }
  cp "$(find $O/t$i -name "*kernel_stats.csv" | head -1)" $O/stats_$i.csv
  cp "$(find $O/t$i -name "*kernel_trace.csv" | head -1)" $O/trace_$i.csv
  echo "== $L"; python3 - "$O/stats_$i.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:10.1f} us")
PY
done
