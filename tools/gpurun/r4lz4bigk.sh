#!/bin/bash
# Kernel times of the LZ4 two-pass decode of one 2 MiB body.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4bigk
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k -o k -- python3 tools/lz4_bench.py --n ${N:-1} --size ${SIZE:-2097152} --steps 3 --no-cpu --no-pipelined --two-pass-only > $O/k.log 2>&1 || { tail -20 $O/k.log; exit 1; }
head -8 $(find $O/k -name "*kernel_stats.csv")
