#!/bin/bash
# CM: execution order of the forked path's small bodies (FSG_SPLIT_WALK 0/2/3)
# x huge-body walk (FSG_CHUNKED_HUGE 0/1), pairs alternating on one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4split2
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread -k "fuzz or large or garbage or wave" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 10 --warmup 2 --verify-sample 16 --workload cm-decompress"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
}
for r in 1 2; do
  for sw in 0 2 3; do
    for ch in 0 1; do run s${sw}_c${ch}_$r FSG_SPLIT_WALK=$sw FSG_CHUNKED_HUGE=$ch || exit 1; done
  done
done
for sw in 0 2; do
  FSG_SPLIT_WALK=$sw timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$sw -o tr -- python3 bench.py --no-cpu-baseline --no-e2e --no-encode --steps 1 --warmup 1 --verify-sample 0 --workload cm-decompress > $O/tr$sw.log 2>&1 || { tail -5 $O/tr$sw.log; exit 1; }
done
