#!/bin/bash
# SQ issue counters (two --pmc passes, 8 SQ counters each) of one workload's
# decode, for the library $LIB (FSG_LIB) with the options in $ENVS
# (FSG_<NAME>=value ..., read by the library at load).
# usage: OUT=gpurun_out/r6sq LIB=build/ab/lib_x.so ENVS="FSG_SPLIT_INDEX=1" WL=c3-decompress bash tools/gpurun/r6sq.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r6sq}
WL=${WL:-c3-decompress}
mkdir -p $O
export FSG_LIB=${LIB:-flare-cpp_amd/lib/libflare_snappy_gpu.so}
for kv in ${ENVS:-}; do export "$kv"; done
Q="--no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $WL"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CU_CYCLES"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/p$i -o sq -- \
    python bench.py --steps 1 --warmup 0 $Q > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  f=$(find $O/p$i -name "*counter_collection.csv" | head -1)
  cp "$f" $O/sq_p$i.csv
  python tools/pmc_sq.py $O/sq_p$i.csv > $O/sq_p$i.txt
done
grep -A12 "index_kernel" $O/sq_p1.txt $O/sq_p2.txt | head -40
