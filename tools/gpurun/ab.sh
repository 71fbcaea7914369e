#!/bin/bash
# A/B of decode builds on one box: parity suite on the candidate, then pairs.
mkdir -p gpurun_out/ab
timeout -k 10 150 python -u -m pytest tests -m gpu -x -q --timeout 60 --timeout-method thread \
  > gpurun_out/ab/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ab/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/ab/pytest_gpu.log
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --pipeline 0 --steps 10 --warmup 2 --verify-sample 16"
run() {  # name lib workload
  FSG_LIB=$2 timeout -k 10 240 $B --workload $3 > gpurun_out/ab/$1_$3.json 2> gpurun_out/ab/$1_$3.err || return 1
  echo "$1 $3 $(python -c "import json,sys;d=json.load(open('gpurun_out/ab/$1_$3.json'));print(d['ms_per_step'], d['value'], d['correct']['oracle_sample_ok'], d['correct']['status_errors'])")"
}
L=flare-cpp_amd/lib/libflare_snappy_gpu.so
for w in ${WLS:-c3-decompress c2-decompress cm-decompress}; do
  run new $L $w && run prev build/ab/lib_prev.so $w && run new2 $L $w && run prev2 build/ab/lib_prev.so $w || exit 1
done
# the candidate's default (pipelined) line
timeout -k 10 240 python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 10 --warmup 2 --verify-sample 16 \
  > gpurun_out/ab/pipe_c3.json 2> gpurun_out/ab/pipe_c3.err || { tail -5 gpurun_out/ab/pipe_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/ab/pipe_c3.json'));print('pipelined c3', d['ms_per_step'], d['value'], d['pipeline'], d['correct'])"
