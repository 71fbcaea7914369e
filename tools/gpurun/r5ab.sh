#!/bin/bash
# In-process A/B of decoder builds (tools/ab_decode.py), then optionally the
# GPU suite.  usage: LIBS="build/ab/lib_a.so build/ab/lib_b.so" WLS="c3" TESTS=1 bash tools/gpurun/r5ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5ab}
mkdir -p $O
for w in ${WLS:-c3}; do
  timeout -k 10 300 python -u tools/ab_decode.py --workload $w --rounds ${ROUNDS:-3} --libs $LIBS > $O/ab_$w.log 2>&1 \
    || { tail -20 $O/ab_$w.log; exit 1; }
  grep -v "^{" $O/ab_$w.log
done
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTARGS:-} \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
