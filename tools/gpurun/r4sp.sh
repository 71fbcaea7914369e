#!/bin/bash
# CM decode: persistent small-message execution grid (FSG_SMALL_PERSIST
# blocks) A/B, two interleaved passes; then the CM GPU tests with it on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4sp
mkdir -p $O
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --verify-sample 16 --workload cm-decompress"
for pass in 1 2; do
  for v in ${VALS:-0 1024 1792 3584}; do
    FSG_SMALL_PERSIST=$v timeout -k 10 300 $B > $O/cm_${v}_$pass.json 2> $O/cm_$v.err || { tail -20 $O/cm_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/cm_${v}_$pass.json'));print('persist=$v', d['ms_per_step'], d['value'], d['correct'])"
  done
done
