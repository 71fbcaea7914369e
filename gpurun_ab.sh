#!/bin/bash
# A/B of exec_kernel window/occupancy variants on one box (C3 decode).
mkdir -p gpurun_out/ab
B="python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 2 --verify-sample 16"
run() {  # name lib workload
  FSG_LIB=$2 timeout -k 10 240 $B --workload $3 > gpurun_out/ab/$1_$3.json 2> gpurun_out/ab/$1_$3.err || return 1
  echo "$1 $3 $(python -c "import json,sys;d=json.load(open('gpurun_out/ab/$1_$3.json'));print(d['ms_per_step'], d['value'])")"
}
run w6 build/ab/lib_w6.so c3-decompress && run w5_6k build/ab/lib_w5_6k.so c3-decompress && run w4_8k build/ab/lib_w4_8k.so c3-decompress &&
run w6b build/ab/lib_w6.so c3-decompress && run w5_6kb build/ab/lib_w5_6k.so c3-decompress && run w4_8kb build/ab/lib_w4_8k.so c3-decompress
