#!/bin/bash
# GPU tests + the C1 echo line + the default bench line.
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  > gpurun_out/r2/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2/pytest_gpu.log
timeout -k 10 300 python bench.py --workload c1-echo --steps 20 > gpurun_out/r2/bench_c1.json 2> gpurun_out/r2/bench_c1.err \
  || { tail -20 gpurun_out/r2/bench_c1.err; exit 1; }
cat gpurun_out/r2/bench_c1.json
