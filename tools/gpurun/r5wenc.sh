#!/bin/bash
# Wave-encoder A/B (tools/ab_encode.py) on the given workloads, then optionally
# the stamps run (tools/wstamps.py, one 64 KiB fragment and a C3-sized batch).
# usage: LIBS="build/ab/lib_a.so build/ab/lib_b.so" WLS="c5 c3w" STAMPS=1 bash tools/gpurun/r5wenc.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5wenc}
mkdir -p $O
for w in ${WLS:-c5}; do
  timeout -k 10 400 python -u tools/ab_encode.py --workload $w --rounds ${ROUNDS:-3} --libs $LIBS > $O/ab_$w.log 2>&1 \
    || { tail -20 $O/ab_$w.log; exit 1; }
  grep -v "^{" $O/ab_$w.log
done
if [ "${STAMPS:-0}" = 1 ]; then
  timeout -k 10 120 python -u tools/wstamps.py 1 65536 > $O/wstamps_1.txt 2>&1 || { tail -20 $O/wstamps_1.txt; exit 1; }
  grep -v amdgpu.ids $O/wstamps_1.txt
  timeout -k 10 200 python -u tools/wstamps.py 4096 65536 > $O/wstamps_4096.txt 2>&1 || { tail -20 $O/wstamps_4096.txt; exit 1; }
  grep -v amdgpu.ids $O/wstamps_4096.txt
fi
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTARGS:-} \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -3 $O/pytest_gpu.log
fi
