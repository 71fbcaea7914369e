#!/bin/bash
# A/B of decode builds on one box: parity suite on the candidate, then C3 pairs.
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/ab/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/ab/pytest_gpu.log
B="python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 2 --verify-sample 16"
run() {  # name lib workload
  FSG_LIB=$2 timeout -k 10 240 $B --workload $3 > gpurun_out/ab/$1_$3.json 2> gpurun_out/ab/$1_$3.err || return 1
  echo "$1 $3 $(python -c "import json,sys;d=json.load(open('gpurun_out/ab/$1_$3.json'));print(d['ms_per_step'], d['value'], d['correct']['oracle_sample_ok'])")"
}
L=flare-cpp_amd/lib/libflare_snappy_gpu.so
for i in 1 2; do
  run new$i $L c3-decompress && run prev$i build/ab/lib_prev.so c3-decompress || exit 1
done
run new $L c2-decompress && run prev build/ab/lib_prev.so c2-decompress
