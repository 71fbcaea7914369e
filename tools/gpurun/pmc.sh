#!/bin/bash
# One PMC pass (SQ counters) over one workload; per-kernel sums printed.
# usage: WL=cm-decompress bash tools/gpurun/pmc.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${WL:-c3-decompress}
O=gpurun_out/pmc_$WL
mkdir -p $O
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $O -o sq -- \
  python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --verify-sample 0 --workload $WL \
  > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python tools/pmc_sq.py $(find $O -name "*counter_collection.csv" | head -1)
