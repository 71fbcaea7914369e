#!/bin/bash
# Two SQ PMC passes (LDS and issue counters) over one workload, each its own run.
# usage: WL=c3-decompress bash tools/gpurun/pmc2.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${WL:-c3-decompress}
O=gpurun_out/pmc2_$WL
mkdir -p $O
P1="SQ_WAVES SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o sq -- \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $WL \
    > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
  python tools/pmc_sq.py $(find $O/p$i -name "*counter_collection.csv" | head -1) | grep -A12 "exec_kernel\|index_kernel"
done
