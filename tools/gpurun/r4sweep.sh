#!/bin/bash
# Snappy decode of 1 GiB of text in bodies of 1-64 KiB (per-message cost), and kernel stats.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4sweep
rm -rf $O; mkdir -p $O
timeout -k 10 400 python tools/size_sweep.py > $O/sweep.jsonl 2> $O/sweep.err || { tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for sz in 1024 65536; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$sz -o k -- python3 tools/size_sweep.py --sizes $sz --steps 3 > $O/k$sz.log 2>&1 || { tail -20 $O/k$sz.log; exit 1; }
  echo "== $sz"; cut -c1-50,150- $(find $O/k$sz -name "*kernel_stats.csv") | grep -v "at::native" | head -8
done
