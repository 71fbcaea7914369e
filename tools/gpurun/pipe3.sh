#!/bin/bash
# Round 3: stream-of-batches decode (lean lane walk beside a persistent
# execution grid) against the serial line, with env knobs, on one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe3; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 20 --warmup 3 --verify-sample 16"
for pass in 1 2; do
  for cfg in ${CFGS:-"p0" "p1" "p1:FSG_EXEC_PERSIST=0" "p1:FSG_EXEC_PERSIST=0:FSG_LEAN_WALK=0" "p1:FSG_EXEC_PERSIST=5"}; do
    p=${cfg%%:*}; envs=$(echo "${cfg#$p}" | tr ':' ' ')
    tag=$(echo "$cfg" | tr ':=' '__')
    env $envs timeout -k 10 240 $B --pipeline ${p#p} --workload ${WL:-c3-decompress} > $O/${tag}_$pass.json 2> $O/${tag}_$pass.err || { tail -5 $O/${tag}_$pass.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${tag}_$pass.json'));pi=d.get('pipeline') or {};print('$cfg', d['ms_per_step'], pi.get('latency_ms_per_batch'), pi.get('serial_ms_per_step'), d['correct'])"
  done
done
