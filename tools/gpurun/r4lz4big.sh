#!/bin/bash
# LZ4 two-pass decode of batches of large bodies (the lane walk's worst case).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4big
rm -rf $O; mkdir -p $O
for cfg in "1 2097152" "16 4194304" "256 262144"; do
  set -- $cfg
  timeout -k 10 300 python tools/lz4_bench.py --n $1 --size $2 --steps 3 --no-cpu --no-pipelined > $O/lz4_$1_$2.json 2> $O/lz4_$1_$2.err || { tail -20 $O/lz4_$1_$2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/lz4_$1_$2.json'));print('$1 x $2', 'one-pass', d['decode']['ms'], 'two-pass', d['decode_two_pass']['ms'], d['decode_two_pass']['roundtrip_ok'], 'ratio', d['ratio'])"
done
