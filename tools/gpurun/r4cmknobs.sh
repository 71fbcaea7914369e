#!/bin/bash
# CM knob sweep at the new defaults (walk-order execution, chunked huge walk).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4cmknobs
rm -rf $O; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 10 --warmup 2 --verify-sample 16 --workload cm-decompress"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['ms_per_step'], d['value'], d['correct']['oracle_sample_ok'], d['correct']['status_errors'])")"
}
for r in 1 2; do
  run def_$r FSG_X=1 || exit 1
  run cls3_$r FSG_SPLIT_CLASS=3 || exit 1
  run cls5_$r FSG_SPLIT_CLASS=5 || exit 1
  run sp1024_$r FSG_SMALL_PERSIST=1024 || exit 1
  run sp3584_$r FSG_SMALL_PERSIST=3584 || exit 1
  run bbf1024_$r FSG_EXEC_BIG_BLOCKS_FORK=1024 || exit 1
  run bbf3584_$r FSG_EXEC_BIG_BLOCKS_FORK=3584 || exit 1
done
