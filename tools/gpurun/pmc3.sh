#!/bin/bash
# L2 / memory-side counters for one workload (two TCC passes).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=${WL:-c3-decompress}
O=gpurun_out/pmc3_$WL
mkdir -p $O
P1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_sum"
P2="TCC_READ_REQ_LATENCY_sum TCC_READ_REQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o sq -- \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $WL \
    > $O/bench$i.log 2>&1 || { tail -20 $O/bench$i.log; exit 1; }
  python tools/pmc_sq.py $(find $O/p$i -name "*counter_collection.csv" | head -1) | grep -A6 "exec_kernel\|index_kernel"
done
