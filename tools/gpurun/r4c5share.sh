#!/bin/bash
# C5 compress: the wave encoder's share of the long units (FSG_ENCODE_WAVE_ALL_MB=0
# applies FSG_ENCODE_WAVE_SHARE), against the default (every long unit on it).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c5share
rm -rf $O; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-e2e --steps 6 --warmup 1 --verify-sample 16 --workload c5-compress"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
}
for r in 1 2; do
  run def_$r FSG_X=1 || exit 1
  for sh in 600 750 900; do run s${sh}_$r FSG_ENCODE_WAVE_ALL_MB=0 FSG_ENCODE_WAVE_SHARE=$sh || exit 1; done
done
