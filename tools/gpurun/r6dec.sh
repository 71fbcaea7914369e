#!/bin/bash
# Decoder: a GPU test subset (-k "$TESTK", or the whole GPU suite with
# TESTS=1), then A/B (tools/ab_decode.py) on the given workloads.
# usage: LIBS="build/ab/lib_a.so build/ab/lib_b.so" WLS="c3 c2 cm" TESTK="decode or fullsize" bash tools/gpurun/r6dec.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r6dec}
mkdir -p $O
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$TESTK" \
    > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
  tail -3 $O/pytest_k.log
fi
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
for w in ${WLS:-}; do
  timeout -k 10 500 python -u tools/ab_decode.py --workload $w --rounds ${ROUNDS:-3} --libs $LIBS > $O/ab_$w.log 2>&1 \
    || { tail -20 $O/ab_$w.log; exit 1; }
  grep -v "^{" $O/ab_$w.log
done
