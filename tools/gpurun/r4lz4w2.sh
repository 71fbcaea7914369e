#!/bin/bash
# LZ4 wave walk, two windows per step: GPU tests, then large-body and small-batch timings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4w2
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "1 2097152" "16 4194304" "256 262144" "1 65536" "256 65536" "65536 65536"; do
  set -- $cfg
  timeout -k 10 300 python tools/lz4_bench.py --n $1 --size $2 --steps 5 --no-cpu --no-pipelined --two-pass-only > $O/lz4_$1_$2.json 2> $O/lz4_$1_$2.err || { tail -20 $O/lz4_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/lz4_$1_$2.json'));print('$1 x $2', 'two-pass', d['decode_two_pass']['ms'], d['decode_two_pass']['roundtrip_ok'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 tools/lz4_bench.py --n 1 --size 2097152 --steps 3 --no-cpu --no-pipelined --two-pass-only > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
cut -c1-60,200- $(find $O/k -name "*kernel_stats.csv") | head -5
