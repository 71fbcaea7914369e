#!/bin/bash
# GPU parity suite (+ optional default bench line), each step under its own time limit.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
grep -h "latches:\|device batches" gpurun_out/pytest_gpu.log | head -5
if [ -n "$BENCH_DEFAULT" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
    || { tail -20 gpurun_out/bench_default.err; exit 1; }
  cat gpurun_out/bench_default.json
fi
for w in ${BENCH_WORKLOADS:-}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-encode --workload $w \
    > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', d['ms_per_step'], d['value'])"
done
