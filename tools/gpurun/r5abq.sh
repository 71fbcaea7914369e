#!/bin/bash
# A/B (tools/ab_decode.py) of $LIBS on $WLS, then per library one SQ counter
# pass over a single decode (exec_kernel / index_kernel lines), then the exec
# phase stamps (tools/stamps.py, libflare_snappy_gpu_stamps.so) if STAMPS=1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5abq}
mkdir -p $O
for w in ${WLS:-c3}; do
  timeout -k 10 400 python -u tools/ab_decode.py --workload $w --rounds ${ROUNDS:-3} --libs $LIBS > $O/ab_$w.log 2>&1 \
    || { tail -20 $O/ab_$w.log; exit 1; }
  grep -v "^{" $O/ab_$w.log
done
if [ "${PMC:-1}" = 1 ]; then
  C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES"
  for l in $LIBS; do
    n=$(basename ${l%%@*} .so)
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$n -o sq -- \
      python tools/ab_decode.py --workload c3 --rounds 1 --steps 1 --warmup 0 --libs $l > $O/pmc_$n.log 2>&1 \
      || { tail -20 $O/pmc_$n.log; exit 1; }
    python tools/pmc_sq.py $(find $O/pmc_$n -name "*counter_collection.csv" | head -1) > $O/sq_$n.txt
    echo "== $n"; grep -A10 "exec_kernel<5>" $O/sq_$n.txt | grep -E "INSTS|LDS_IDX|WAVE_CYC|per wave"
  done
fi
if [ "${STAMPS:-0}" = 1 ]; then
  timeout -k 10 200 python tools/stamps.py text > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
  cat $O/stamps.txt
fi
