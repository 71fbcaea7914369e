#!/bin/bash
# Encoder A/B (tools/ab_encode.py) on the given workloads, then optionally a
# GPU test subset (-k "$TESTK") or the whole GPU suite (TESTS=1).
# usage: LIBS="build/ab/lib_a.so build/ab/lib_b.so@opt=v" WLS="c3 c5" TESTK="partial or iovec" bash tools/gpurun/r6enc.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r6enc}
mkdir -p $O
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" \
    > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
  tail -3 $O/pytest_k.log
fi
for w in ${WLS:-}; do
  timeout -k 10 500 python -u tools/ab_encode.py --workload $w --rounds ${ROUNDS:-3} --libs $LIBS > $O/ab_$w.log 2>&1 \
    || { tail -20 $O/ab_$w.log; exit 1; }
  grep -v "^{" $O/ab_$w.log
done
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
