#!/bin/bash
# LZ4 small batches: wave walk from 2 KiB (default) vs the lane walk (FSG_L4_BIG_MIN=65536).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4sm
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "1 65536" "1 8192" "64 16384" "256 65536"; do
  set -- $cfg
  for t in def 65536; do
    if [ $t = def ]; then unset FSG_L4_BIG_MIN; else export FSG_L4_BIG_MIN=$t; fi
    timeout -k 10 300 python tools/lz4_bench.py --n $1 --size $2 --steps 20 --no-cpu --no-pipelined --two-pass-only > $O/s_$1_$2_$t.json 2> $O/s_$1_$2_$t.err || { tail -20 $O/s_$1_$2_$t.err; exit 1; }
    python -c "import json;d=json.load(open('$O/s_$1_$2_$t.json'));print('$1 x $2 big_min=$t', d['decode_two_pass']['ms'], d['decode_two_pass']['roundtrip_ok'])"
  done
done
