#!/bin/bash
# A/B of encode builds on one box: parity suite on the candidate, then compress pairs.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ab/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/ab/pytest_gpu.log
B="python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 --verify-sample 16"
run() {  # name lib workload
  FSG_LIB=$2 timeout -k 10 240 $B --workload $3 > gpurun_out/ab/$1_$3.json 2> gpurun_out/ab/$1_$3.err || return 1
  echo "$1 $3 $(python -c "import json,sys;d=json.load(open('gpurun_out/ab/$1_$3.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
}
L=flare-cpp_amd/lib/libflare_snappy_gpu.so
run new $L c3-compress && run prev build/ab/lib_prev.so c3-compress &&
run new $L c5-compress && run prev build/ab/lib_prev.so c5-compress
