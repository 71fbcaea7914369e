#!/bin/bash
# Forked-path GPU tests (persistent small grid included) + CM bench at defaults.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4t2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "fuzz or garbage or large_message or wave_encoder" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --verify-sample 16 --workload cm-decompress > $O/cm.json 2> $O/cm.err || { tail -20 $O/cm.err; exit 1; }
python -c "import json;d=json.load(open('$O/cm.json'));print('cm', d['ms_per_step'], d['value'], d['correct'])"
