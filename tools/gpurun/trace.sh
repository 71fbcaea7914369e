#!/bin/bash
# Kernel timeline of a few steps of one workload (rocprofv3 --kernel-trace).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${WL:-cm-decompress}; O=gpurun_out/trace_$WL; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o tr -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $WL \
  > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 tools/timeline.py $(find $O -name "*kernel_trace.csv" | head -1) > $O/timeline.txt && tail -40 $O/timeline.txt
