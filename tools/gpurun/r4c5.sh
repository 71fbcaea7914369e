#!/bin/bash
# C5 compress: wave-encoder minimum message size (FSG_ENCODE_WAVE_MIN) A/B,
# two interleaved passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c5
mkdir -p $O
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --verify-sample 16 --workload c5-compress"
for pass in 1 2; do
  for v in ${VALS:-16384 24576 32768 49152}; do
    FSG_ENCODE_WAVE_MIN=$v timeout -k 10 300 $B > $O/c5_${v}_$pass.json 2> $O/c5_$v.err || { tail -20 $O/c5_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c5_${v}_$pass.json'));print('wave_min=$v', d['ms_per_step'], d['value'], d['correct'])"
  done
done
