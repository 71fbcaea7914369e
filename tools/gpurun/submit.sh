#!/bin/bash
# Submits one gpurun call; when the pool reports no free slot or box (status
# "transient": nothing ran, nothing was charged) it waits two minutes and
# submits the same call again, at most 6 times.  A call that ran -- whatever
# its exit code -- is never resubmitted.
# usage: bash tools/gpurun/submit.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  grep -q "status=transient" "$LOG" || exit $rc
  sleep 120
done
exit $rc
