#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5tiny2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "${TK:-tiny or fuzz_against or garbage}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
L=flare-cpp_amd/lib/libflare_snappy_gpu.so
timeout -k 10 400 python -u tools/ab_decode.py --workload cm --rounds 3 --libs $L@tiny_pass=1 $L@tiny_pass=0 > $O/ab_cm.log 2>&1 \
  || { tail -20 $O/ab_cm.log; exit 1; }
grep -v "^{" $O/ab_cm.log
OUT=$O/kt LIBS="$L@tiny_pass=1" bash tools/gpurun/r5ktrace.sh > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
grep -E "tiny|index_kernel|exec_kernel|index_big|chunk_spec" $O/kt.log
