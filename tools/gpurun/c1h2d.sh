#!/bin/bash
# C1 echo line (three runs, each its own process) and the C3 end-to-end leg
# under rocprofv3 --memory-copy-trace (the serial H2D's copies next to the
# diagnostic ones).  usage: bash tools/gpurun/c1h2d.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c1h2d
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload c1-echo --steps 20 > $O/bench_c1_$i.json 2> $O/bench_c1_$i.err \
    || { tail -20 $O/bench_c1_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c1_$i.json'));print('c1', d['value'], d['p50_us'], {k:v['qps'] for k,v in d['modes'].items()}, d['cpu_baseline']['value'])"
done
mkdir -p $O/mc
timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d $O/mc -o mc -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-encode --verify-sample 0 > $O/mc/bench.json 2> $O/mc/bench.err \
  || { tail -20 $O/mc/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/mc/bench.json'));print(json.dumps(d.get('end_to_end'))[:1500])"
ls $O/mc/*/ 2>/dev/null | head; f=$(find $O/mc -name "*memory_copy_trace.csv" | head -1); head -3 "$f"; wc -l "$f"
