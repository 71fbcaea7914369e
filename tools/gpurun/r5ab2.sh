#!/bin/bash
# A/B + WRITE_SIZE of the index pass for the super-group stores
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5ab2}
mkdir -p $O
for w in ${WLS:-c3}; do
  timeout -k 10 400 python -u tools/ab_decode.py --workload $w --rounds ${ROUNDS:-3} --libs $LIBS > $O/ab_$w.log 2>&1 \
    || { tail -20 $O/ab_$w.log; exit 1; }
  grep -v "^{" $O/ab_$w.log
done
for l in $WLIBS; do
  n=$(basename $l .so)
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o w -- \
    python tools/ab_decode.py --workload c3 --rounds 1 --steps 1 --warmup 0 --libs $l > $O/w_$n.log 2>&1 \
    || { tail -20 $O/w_$n.log; exit 1; }
  python tools/pmc_sq.py $(find $O/w_$n -name "*counter_collection.csv" | head -1) > $O/w_$n.txt
  echo "== $n"; grep -A2 "index_kernel\|exec_kernel<5>" $O/w_$n.txt
done
