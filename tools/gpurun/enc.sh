#!/bin/bash
# Encode variants on C3 compress: v3 at several lane counts (FSG_ENCODE_LANES),
# and the LDS-table v1 encoder.
mkdir -p gpurun_out/enc
B="python bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 --verify-sample 16 --workload c3-compress"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 300 $B > gpurun_out/enc/$n.json 2> gpurun_out/enc/$n.err || { tail -5 gpurun_out/enc/$n.err; return 1; }
  echo "$n $(python -c "import json;d=json.load(open('gpurun_out/enc/$n.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
}
run v3 FSG_ENCODE_KERNEL=3 && run v3_l8192 FSG_ENCODE_LANES=8192 && run v3_l16384 FSG_ENCODE_LANES=16384 \
  && run v3_l32768 FSG_ENCODE_LANES=32768 && run v3_l4096 FSG_ENCODE_LANES=4096 && run v1 FSG_ENCODE_KERNEL=1
