#!/bin/bash
# Split lane walk (forked path): GPU parity suite, then CM with FSG_SPLIT_WALK
# off / on and a split-class sweep, pairs alternating on one box.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4split
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --steps 10 --warmup 2 --verify-sample 16 --workload cm-decompress"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 240 $B > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; return 1; }
  echo "$name $(python -c "import json;d=json.load(open('$O/$name.json'));print(d['ms_per_step'], d['value'], d['correct'])")"
}
run off1 FSG_SPLIT_WALK=0 && run on1 FSG_SPLIT_WALK=1 && run off2 FSG_SPLIT_WALK=0 && run on2 FSG_SPLIT_WALK=1 || exit 1
for c in 3 5 6; do run c$c FSG_SPLIT_WALK=1 FSG_SPLIT_CLASS=$c || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o tr -- python3 bench.py --no-cpu-baseline --no-e2e --no-encode --steps 1 --warmup 1 --verify-sample 0 --workload cm-decompress > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
ls $O/tr/*/ 2>/dev/null | head -3
