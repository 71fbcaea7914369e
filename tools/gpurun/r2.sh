#!/bin/bash
# Round-2 evidence at HEAD: GPU parity suite, the default bench line, kernel
# stats for C3 and CM decode, and the FETCH_SIZE / WRITE_SIZE passes for C3
# decode (each its own rocprofv3 run).  Optional probes first (PROBES=1).
# usage: bash tools/gpurun/r2.sh   (outputs under gpurun_out/r2/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r2}
mkdir -p $O
if [ -n "$PROBES" ]; then
  for p in $PROBES; do
    timeout -k 10 120 build/$p > $O/$p.txt 2>&1 || { cat $O/$p.txt; exit 1; }
    cat $O/$p.txt
  done
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
  echo smoke ok
fi
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
for w in ${BENCH_WORKLOADS:-}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-encode --workload $w \
    > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
for WL in c3-decompress cm-decompress; do
  mkdir -p $O/prof_$WL
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$WL -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $WL \
    > $O/prof_$WL/bench.log 2>&1 || { tail -20 $O/prof_$WL/bench.log; exit 1; }
  f=$(find $O/prof_$WL -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_$WL.csv
  cut -d, -f1-8 $O/kernel_stats_$WL.csv | head -8
done
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$C -o pmc -- \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload c3-decompress \
    > $O/pmc_$C.log 2>&1 || { tail -20 $O/pmc_$C.log; exit 1; }
  cp $(find $O/pmc_$C -name "*counter_collection.csv" | head -1) $O/pmc_${C}_c3d.csv
done
echo done
