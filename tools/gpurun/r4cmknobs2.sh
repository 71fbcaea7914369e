#!/bin/bash
# CM: small grid 3,584 + forked large grid 1,024 together vs the defaults.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4cmknobs2
rm -rf $O; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 10 --warmup 2 --verify-sample 16 --workload cm-decompress"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['ms_per_step'], d['value'], d['correct']['oracle_sample_ok'], d['correct']['status_errors'])")"
}
for r in 1 2 3 4; do
  run def_$r FSG_X=1 && run both_$r FSG_SMALL_PERSIST=3584 FSG_EXEC_BIG_BLOCKS_FORK=1024 || exit 1
done
