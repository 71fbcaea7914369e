#!/bin/bash
# Launch-order effect: kernel traces of C3 decode steps with and without the
# trailing fallback launch (FSG_DIAG_NO_TAIL=1); per-kernel start gaps and
# durations by step.  usage: bash tools/gpurun/tail.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in tail notail; do  # FSG_LIB in the environment selects an A/B build
  O=gpurun_out/tail/$v
  mkdir -p $O
  if [ $v = notail ]; then export FSG_DIAG_NO_TAIL=1; else unset FSG_DIAG_NO_TAIL; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
    python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload c3-decompress \
    > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
  cp $(find $O -name "*kernel_trace.csv" | head -1) gpurun_out/tail/trace_$v.csv
  python -c "
import json
for l in open('$O/bench.log'):
    if l.startswith('{'): print('$v', json.loads(l)['ms_per_step'])"
done
