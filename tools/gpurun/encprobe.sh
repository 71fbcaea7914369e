#!/bin/bash
mkdir -p gpurun_out/enc
B="python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 --verify-sample 8"
for k in 0 1; do
  for spec in "c5-compress 262144" "c3-compress 1024" "c3-compress 4096"; do
    set -- $spec
    timeout -k 10 300 $B --workload $1 --n-msgs $2 --encode-kernel $k > gpurun_out/enc/$1_$2_$k.json 2> gpurun_out/enc/$1_$2_$k.err || { tail -5 gpurun_out/enc/$1_$2_$k.err; exit 1; }
    echo "k=$k $1 n=$2 $(python -c "import json;d=json.load(open('gpurun_out/enc/$1_$2_$k.json'));print(d['ms_per_step'], d['value'])")"
  done
done
