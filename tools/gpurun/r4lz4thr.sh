#!/bin/bash
# LZ4 C3 decode with the wave walk for every block (FSG_L4_BIG_MIN) vs the lane walk.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4thr
rm -rf $O; mkdir -p $O
for t in 65536 16384 65536 16384; do
  FSG_L4_BIG_MIN=$t timeout -k 10 300 python tools/lz4_bench.py --steps 4 --no-cpu --no-pipelined --two-pass-only > $O/c3_$t.json 2> $O/c3_$t.err || { tail -20 $O/c3_$t.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c3_$t.json'));print('big_min $t', d['decode_two_pass']['ms'], d['decode_two_pass']['roundtrip_ok'])"
done
FSG_L4_BIG_MIN=16384 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 tools/lz4_bench.py --steps 3 --no-cpu --no-pipelined --two-pass-only > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
cut -c1-60,200- $(find $O/k -name "*kernel_stats.csv") | head -6
