#!/bin/bash
# Instruction accounting for the exec pass: SQ counters of diagnostic builds
# that skip a phase (wrong output, counters only) next to the real one, and
# the v5 phase stamps.  usage: bash tools/gpurun/acct.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/acct
mkdir -p $O
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --pipeline 0 --verify-sample 0 --workload c3-decompress"
for lib in ${ACCT_LIBS:-cur nob noa noab}; do
  FSG_LIB=build/ab/lib_$lib.so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    --output-format csv -d $O/sq_$lib -o sq -- $B > $O/sq_$lib.log 2>&1 || { tail -20 $O/sq_$lib.log; exit 1; }
  python tools/pmc_sq.py $(find $O/sq_$lib -name "*counter_collection.csv" | head -1) > $O/sq_$lib.txt
  echo "== $lib $(grep -A10 'exec_kernel' $O/sq_$lib.txt | grep 'per wave')"
done
timeout -k 10 120 python tools/stamps.py > $O/stamps5.txt 2>&1 || { tail -20 $O/stamps5.txt; exit 1; }
cat $O/stamps5.txt
