#!/bin/bash
# GPU parity suite + short bench lines, each step under its own time limit.
mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest tests -m gpu -x -v --timeout 60 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for w in ${BENCH_WORKLOADS:-c3-decompress}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --workload $w \
    > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', d['ms_per_step'], d['value'])"
done
