#!/bin/bash
# Kernel-trace stats per A/B library: LIBS="a b" WLS="c3-decompress" bash tools/gpurun/abprof.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in ${WLS:-c3-decompress}; do
  for n in $LIBS; do
    O=gpurun_out/abprof/${n}_$w
    mkdir -p $O
    FSG_LIB=build/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
      python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $w \
      > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
    f=$(find $O -name "*kernel_stats.csv" | head -1)
    python -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'fsg::' in r['Name']: print('$n $w', r['Name'].split('(')[0].replace('void ',''), r['Calls'], round(float(r['AverageNs'])/1e6,4))"
  done
done
