#!/bin/bash
# LZ4 encode A/B: GPU parity, then tools/lz4_bench.py (encode + two-pass
# decode) per library (current + build/ab/lib_<name>.so per argument).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in cur "$@"; do
  L=flare-cpp_amd/lib/libflare_snappy_gpu.so
  [ "$v" != cur ] && L=build/ab/lib_$v.so
  FSG_LIB=$L timeout -k 10 300 python tools/lz4_bench.py --steps 3 --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', d['encode'], d['decode_two_pass']['ms'], d['oracle_sample_ok'])"
done
