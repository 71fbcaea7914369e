#!/bin/bash
# Round 3: GPU parity suite, smoke, then bench lines (default = pipelined
# C3 decode; BENCH_WORKLOADS adds lines) with and without the pipeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
  echo smoke ok
fi
for w in ${BENCH_WORKLOADS:-c3-decompress c2-decompress cm-decompress}; do
  for p in 1 0; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-encode --pipeline $p \
      --workload $w > $O/bench_${w}_p$p.json 2> $O/bench_${w}_p$p.err || { tail -20 $O/bench_${w}_p$p.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${w}_p$p.json'));print('$w pipe=$p', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('pipeline'), d['correct'])"
  done
done
