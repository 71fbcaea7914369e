#!/bin/bash
# A/B of libraries (current + build/ab/lib_<name>.so per argument) on the
# decode workloads (WLS), two interleaved passes; GPU parity tests first
# (TESTS=1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4ab
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -k "${TESTK:-not lz4}" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
Q="--no-cpu-baseline --no-e2e --no-encode --verify-sample 16"
for pass in 1 2; do
  for v in cur "$@"; do
    L=flare-cpp_amd/lib/libflare_snappy_gpu.so
    [ "$v" != cur ] && L=build/ab/lib_$v.so
    for w in ${WLS:-c3-decompress c2-decompress cm-decompress}; do
      FSG_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 $Q --workload $w > $O/${v}_${w}_$pass.json 2> $O/${v}_$w.err || { tail -20 $O/${v}_$w.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${v}_${w}_$pass.json'));print('$v $w', d['ms_per_step'], d['correct']['roundtrip_ok'])"
    done
  done
done
