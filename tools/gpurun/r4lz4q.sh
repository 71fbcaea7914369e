#!/bin/bash
# LZ4 two-pass decode: SQ counters per kernel (one --pmc pass per library:
# the current one and build/ab/lib_<name>.so for each argument).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4q
mkdir -p $O
for v in cur "$@"; do
  L=flare-cpp_amd/lib/libflare_snappy_gpu.so
  [ "$v" != cur ] && L=build/ab/lib_$v.so
  FSG_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/sq_$v -o sq -- python3 tools/lz4_bench.py --steps 1 --two-pass-only --no-cpu > $O/sq_$v.log 2>&1 || { tail -20 $O/sq_$v.log; exit 1; }
  echo "== $v"
  python3 tools/pmc_sq.py $(find $O/sq_$v -name "*counter_collection.csv" | head -1) | grep -A12 lz4_
done
