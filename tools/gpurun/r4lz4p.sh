#!/bin/bash
# LZ4 two-pass decode: kernel split (rocprofv3 stats) for the current library
# and for A/B variants build/ab/lib_<name>.so given as arguments.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4p
mkdir -p $O
for v in cur "$@"; do
  L=flare-cpp_amd/lib/libflare_snappy_gpu.so
  [ "$v" != cur ] && L=build/ab/lib_$v.so
  FSG_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 tools/lz4_bench.py --steps 5 --two-pass-only --no-cpu > $O/bench_$v.json 2> $O/prof_$v.log || { tail -20 $O/prof_$v.log; exit 1; }
  echo "== $v: $(python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print(d['decode_two_pass'])")"
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'lz4' in r['Name']: print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
