#!/bin/bash
mkdir -p gpurun_out/enc2
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variants or golden or randomized or split_message" > gpurun_out/enc2/pytest.log 2>&1 || { tail -30 gpurun_out/enc2/pytest.log; exit 1; }
tail -1 gpurun_out/enc2/pytest.log
B="python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 --verify-sample 8"
for spec in "c3-compress 1024 1" "c3-compress 4096 1" "c5-compress 262144 1" "c3-compress 65536 1"; do
  set -- $spec
  timeout -k 10 300 $B --workload $1 --n-msgs $2 --encode-kernel $3 > gpurun_out/enc2/$1_$2_$3.json 2> gpurun_out/enc2/$1_$2_$3.err || { tail -5 gpurun_out/enc2/$1_$2_$3.err; exit 1; }
  echo "k=$3 $1 n=$2 $(python -c "import json;d=json.load(open('gpurun_out/enc2/$1_$2_$3.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
done
