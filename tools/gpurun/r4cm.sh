#!/bin/bash
# Round 4: chunked pass 1b for the huge messages -- parity (large-message
# tests, garbage workspace, segments), CM A/B, CM timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4cm
mkdir -p $O
FSG_CHUNKED_HUGE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "large_message or garbage or segments or config_digests" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --verify-sample 16 --workload cm-decompress"
for pass in 1 2; do
  for c in 1 0; do
    FSG_CHUNKED_HUGE=$c timeout -k 10 300 $B > $O/cm_${c}_${pass}.json 2> $O/cm_${c}.err || { tail -20 $O/cm_${c}.err; exit 1; }
    python -c "import json;d=json.load(open('$O/cm_${c}_${pass}.json'));print('cm chunked=$c', d['ms_per_step'], d['value'], d['correct'])"
  done
done
FSG_CHUNKED_HUGE=1 WL=cm-decompress bash tools/gpurun/trace.sh
