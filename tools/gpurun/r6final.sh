#!/bin/bash
# Round-6 evidence at HEAD: GPU parity suite + smoke, the default bench line,
# a bench line per workload, rocprofv3 kernel stats per workload, and the
# FETCH_SIZE / WRITE_SIZE passes (one --pmc run each) summarised into
# profiles/pmc_<workload>.json.  PART=tests|bench|pmc selects a part (default all).
# usage: OUT=gpurun_out/r6final PART=... bash tools/gpurun/r6final.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r6final}
P=${PART:-all}
mkdir -p $O
WLS=${WLS:-"c3-decompress c2-decompress cm-decompress c3-compress c5-compress"}
Q="--no-cpu-baseline --no-e2e --no-encode"
if [ $P = all -o $P = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
  echo smoke ok
fi
if [ $P = all -o $P = bench ]; then
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
    || { tail -20 $O/bench_default.err; exit 1; }
  cat $O/bench_default.json
  for w in $WLS; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 $Q --verify-sample 16 --workload $w \
      > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['ms_per_step'], d['value'], d['roofline']['frac'], d['correct'])"
  done
  for w in $WLS; do
    mkdir -p $O/prof_$w
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
      python bench.py --steps 3 --warmup 1 $Q --verify-sample 0 --workload $w > $O/prof_$w/bench.log 2>&1 \
      || { tail -20 $O/prof_$w/bench.log; exit 1; }
    cp "$(find $O/prof_$w -name "*kernel_stats.csv" | head -1)" $O/kernel_stats_$w.csv
    echo "== $w"; cut -d, -f1-4 $O/kernel_stats_$w.csv | head -6
  done
  timeout -k 10 300 python tools/lz4_bench.py --steps 5 > $O/lz4_bench.json 2> $O/lz4_bench.err \
    || { tail -20 $O/lz4_bench.err; exit 1; }
  cat $O/lz4_bench.json
fi
if [ $P = all -o $P = pmc ]; then
  for w in $WLS; do
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${C}_$w -o pmc -- \
        python bench.py --steps 1 --warmup 0 $Q --verify-sample 0 --workload $w > $O/pmc_${C}_$w.log 2>&1 \
        || { tail -20 $O/pmc_${C}_$w.log; exit 1; }
      cp "$(find $O/pmc_${C}_$w -name "*counter_collection.csv" | head -1)" $O/pmc_${C}_$w.csv
    done
    algo=$(python -c "import json;print([json.loads(l) for l in open('$O/pmc_FETCH_SIZE_$w.log') if l.startswith('{\"metric')][-1]['roofline']['algorithmic_bytes_per_launch'])")
    python tools/pmc_summary.py $w $O/pmc_FETCH_SIZE_$w.csv $O/pmc_WRITE_SIZE_$w.csv $algo > $O/pmc_$w.json \
      || { echo "summary failed: $w"; exit 1; }
    python -c "import json;d=json.load(open('$O/pmc_$w.json'));print('$w traffic', d['traffic_bytes_per_launch'], 'algo', d['algorithmic_bytes_per_launch'], d['traffic_over_algorithmic'])"
  done
fi
echo done
