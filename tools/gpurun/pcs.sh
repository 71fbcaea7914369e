#!/bin/bash
# PC sampling (host trap, beta) of one C3 decode step: where the exec pass's
# issue slots go, per instruction.  usage: V=5 bash tools/gpurun/pcs.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pcs${V:-5}
mkdir -p $O
FSG_DECODE_KERNEL=${V:-5} timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
  --pc-sampling-unit time --pc-sampling-interval ${IV:-1} --output-format csv -d $O -o pcs -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-encode --pipeline 0 --verify-sample 0 \
  > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
find $O -name "*.csv" | head
for f in $(find $O -name "*.csv"); do echo "== $f"; head -3 $f; wc -l $f; done
