#!/bin/bash
# Kernel-trace stats for one workload: rocprofv3 --kernel-trace --stats.
# usage: WL=cm-decompress bash tools/gpurun/prof.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${WL:-c3-decompress}
mkdir -p gpurun_out/prof_$WL
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$WL -o run -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --verify-sample 0 --workload $WL \
  > gpurun_out/prof_$WL/bench.log 2>&1 || { tail -20 gpurun_out/prof_$WL/bench.log; exit 1; }
f=$(find gpurun_out/prof_$WL -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/prof_$WL/kernel_stats.csv
cut -d, -f1-8 gpurun_out/prof_$WL/kernel_stats.csv | head -12
