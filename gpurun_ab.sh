#!/bin/bash
# A/B of encode builds on one box (compress pairs).
mkdir -p gpurun_out/ab
B="python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 --verify-sample 16"
run() {  # name lib workload
  FSG_LIB=$2 timeout -k 10 240 $B --workload $3 > gpurun_out/ab/$1_$3.json 2> gpurun_out/ab/$1_$3.err || return 1
  echo "$1 $3 $(python -c "import json,sys;d=json.load(open('gpurun_out/ab/$1_$3.json'));print(d['ms_per_step'], d['value'], d['correct']['oracle_sample_ok'], d['correct']['roundtrip_ok'])")"
}
for w in c3-compress c5-compress; do
  for v in prev k1 k3 k3p1 k3p2 k4p2; do run $v build/ab/lib_$v.so $w || exit 1; done
done
