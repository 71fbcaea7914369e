#!/bin/bash
# Round 3: exec v4 (pieces) vs v5 (tag per lane) on one box -- A/B pairs,
# SQ instruction counters and kernel stats for each.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/v5
mkdir -p $O
LIBS=${LIBS:-"cur@FSG_DECODE_KERNEL=4 cur@FSG_DECODE_KERNEL=5"} WLS=${WLS:-c3-decompress} bash tools/gpurun/abn.sh || exit 1
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-encode --pipeline 0 --verify-sample 0 --workload c3-decompress"
for v in ${PMCV:-4 5}; do
  FSG_DECODE_KERNEL=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d $O/sq$v -o sq -- $B > $O/sq$v.log 2>&1 || { tail -20 $O/sq$v.log; exit 1; }
  echo "== exec v$v"; python tools/pmc_sq.py $(find $O/sq$v -name "*counter_collection.csv" | head -1) | head -30
done
