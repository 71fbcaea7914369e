#!/bin/bash
# CM: new defaults (walk-order execution, chunked huge walk) vs the previous ones.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4split3
rm -rf $O; mkdir -p $O
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 10 --warmup 2 --verify-sample 16 --workload cm-decompress"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
}
for r in 1 2 3; do
  run new_$r FSG_DECODE_FORK=1 && run old_$r FSG_SPLIT_WALK=0 FSG_CHUNKED_HUGE=0 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --no-cpu-baseline --no-e2e --no-encode --steps 1 --warmup 1 --verify-sample 0 --workload cm-decompress > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
