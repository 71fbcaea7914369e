#!/bin/bash
# Wave encoder phase stamps for one-message batches (stage on / off).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4ws1
rm -rf $O; mkdir -p $O
for s in 1 0; do
  for sz in 4096 65536; do
    echo "== stage=$s size=$sz"
    FSG_ENCODE_WAVE_STAGE=$s timeout -k 10 120 python tools/wstamps.py 1 $sz > $O/s${s}_$sz.txt 2>&1 || { tail -20 $O/s${s}_$sz.txt; exit 1; }
    cat $O/s${s}_$sz.txt
  done
done
