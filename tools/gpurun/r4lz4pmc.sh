#!/bin/bash
# LZ4 C3 two-pass decode: FETCH_SIZE / WRITE_SIZE per kernel (one --pmc pass each).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4pmc
rm -rf $O; mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/$C -o p -- python3 tools/lz4_bench.py --steps 1 --two-pass-only --no-cpu --no-pipelined > $O/$C.log 2>&1 || { tail -20 $O/$C.log; exit 1; }
  cp "$(find $O/$C -name "*counter_collection.csv" | head -1)" $O/$C.csv
  echo "== $C"; python3 tools/pmc_sq.py $O/$C.csv | grep -A2 "lz4_"
done
