#!/bin/bash
# Kernel trace (per-dispatch rows + stats) of one bench workload.
# usage: WL=c5-compress bash tools/gpurun/ktrace.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ktrace_${WL:-c5-compress}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --pipeline 0 \
  --verify-sample 4 --workload ${WL:-c5-compress} > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cut -d, -f1-8 "$(find $O -name "*kernel_stats.csv" | head -1)" | head -12
