#!/bin/bash
# Round 5: SQ issue counters of the C3 decode kernels at HEAD (two --pmc
# passes, 8 SQ counters each) plus kernel stats, for the per-group budget.
# usage: OUT=gpurun_out/r5sq WL=c3-decompress bash tools/gpurun/r5sq.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5sq}
WL=${WL:-c3-decompress}
mkdir -p $O
Q="--no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $WL"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_BUSY_CU_CYCLES"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o sq -- \
    python bench.py --steps 1 --warmup 0 $Q > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  f=$(find $O/p$i -name "*counter_collection.csv" | head -1)
  cp "$f" $O/sq_p$i.csv
  python tools/pmc_sq.py $O/sq_p$i.csv > $O/sq_p$i.txt
done
mkdir -p $O/ks
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o run -- \
  python bench.py --steps 5 --warmup 2 $Q > $O/ks/bench.log 2>&1 || { tail -20 $O/ks/bench.log; exit 1; }
cp "$(find $O/ks -name "*kernel_stats.csv" | head -1)" $O/kernel_stats.csv
cut -d, -f1-4 $O/kernel_stats.csv | head -8
cat $O/sq_p1.txt $O/sq_p2.txt | head -60
