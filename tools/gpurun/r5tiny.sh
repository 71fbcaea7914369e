#!/bin/bash
# Tiny-body pass: its parity tests, then CM A/B (tiny_pass on/off) and C3 A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/r5tiny}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "${TK:-tiny or fuzz or garbage or config_digests}" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
L=flare-cpp_amd/lib/libflare_snappy_gpu.so
timeout -k 10 400 python -u tools/ab_decode.py --workload cm --rounds 3 --libs $L@tiny_pass=1 $L@tiny_pass=0 > $O/ab_cm.log 2>&1 \
  || { tail -20 $O/ab_cm.log; exit 1; }
grep -v "^{" $O/ab_cm.log
timeout -k 10 400 python -u tools/ab_decode.py --workload c3 --rounds 3 --libs build/ab/lib_super.so build/ab/lib_nosuper.so > $O/ab_c3.log 2>&1 \
  || { tail -20 $O/ab_c3.log; exit 1; }
grep -v "^{" $O/ab_c3.log
