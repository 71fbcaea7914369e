#!/bin/bash
# FETCH_SIZE calibration of the exec pass's far-load pattern
# (tools/probes/fetch_probe.hip, built in-tree as build/fetch_probe), one
# --pmc pass per counter set, plus the list of the TCC_EA0 read counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r6fetch}
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -E "TCC_EA0_RD|TCC_EA_RD|TCC_BUBBLE|TCC_REQ|TCC_HIT|TCC_MISS" $O/avail.txt | head -40 > $O/avail_tcc.txt || true
for C in "FETCH_SIZE" ${EXTRA:-}; do
  tag=$(echo "$C" | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/p_$tag -o fp -- ./build/fetch_probe > $O/p_$tag.log 2>&1 \
    || { tail -20 $O/p_$tag.log; exit 1; }
  cp "$(find $O/p_$tag -name "*counter_collection.csv" | head -1)" $O/fp_$tag.csv
done
cat $O/avail_tcc.txt
