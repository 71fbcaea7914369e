#!/bin/bash
# SQ counters of the Snappy exec pass on 1 GiB of text in 1 KiB vs 16 KiB bodies.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4sweepq
rm -rf $O; mkdir -p $O
for sz in 1024 16384; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/q$sz -o q -- python3 tools/size_sweep.py --sizes $sz --steps 1 > $O/q$sz.log 2>&1 || { tail -20 $O/q$sz.log; exit 1; }
  echo "== $sz"; python3 tools/pmc_sq.py $(find $O/q$sz -name "*counter_collection.csv" | head -1) | grep -A11 "exec_kernel\|index_kernel"
done
