#!/bin/bash
# Kernel stats of the LZ4 C3 two-pass decode (rocprofv3 --kernel-trace --stats).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4k
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 tools/lz4_bench.py --steps 5 --two-pass-only --no-cpu --no-pipelined > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
cp "$(find $O/k -name "*kernel_stats.csv" | head -1)" $O/kernel_stats_lz4-c3-decompress.csv
cut -d, -f1-4 $O/kernel_stats_lz4-c3-decompress.csv | sed 's/(unsigned[^"]*//' | head -8
grep decode_two_pass $O/k.log | head -2 || true
