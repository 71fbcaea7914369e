#!/bin/bash
# Round-3 evidence at HEAD: GPU parity suite, smoke, the default bench line,
# kernel stats (C3, CM decode; C3 encode), SQ instruction and LDS counter
# passes on C3 decode, FETCH/WRITE passes (C3 decode and encode), exec phase
# stamps.  Each profiler pass is its own run.  usage: OUT=gpurun_out/x bash tools/gpurun/head3.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/head3}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
  echo smoke ok
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err \
    || { tail -20 $O/bench_default.err; exit 1; }
  cat $O/bench_default.json
fi
Q="--no-cpu-baseline --no-e2e --no-encode --verify-sample 0"
for w in ${BENCH_WORKLOADS:-}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 $Q --workload $w \
    > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$w.json'));print('$w', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
for WL in ${KSTATS:-c3-decompress cm-decompress c3-compress}; do
  mkdir -p $O/prof_$WL
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$WL -o run -- \
    python bench.py --steps 3 --warmup 1 $Q --workload $WL > $O/prof_$WL/bench.log 2>&1 \
    || { tail -20 $O/prof_$WL/bench.log; exit 1; }
  cp "$(find $O/prof_$WL -name "*kernel_stats.csv" | head -1)" $O/kernel_stats_$WL.csv
  cut -d, -f1-8 $O/kernel_stats_$WL.csv | head -8
done
B1="python bench.py --steps 1 --warmup 0 $Q"
pmc() {  # name workload counters...
  local name=$1 wl=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $O/pmc_$name -o pmc -- \
    $B1 --workload $wl > $O/pmc_$name.log 2>&1 || { tail -20 $O/pmc_$name.log; return 1; }
  cp "$(find $O/pmc_$name -name "*counter_collection.csv" | head -1)" $O/pmc_$name.csv
  python tools/pmc_sq.py $O/pmc_$name.csv > $O/pmc_$name.txt
}
if [ -z "$SKIP_PMC" ]; then
  pmc sq_c3d c3-decompress SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit 1
  pmc lds_c3d c3-decompress SQ_WAVES SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS || exit 1
  for C in FETCH_SIZE WRITE_SIZE; do
    pmc ${C}_c3d c3-decompress $C || exit 1
    pmc ${C}_c3c c3-compress $C || exit 1
  done
  grep -A12 "exec_kernel\|index_kernel" $O/pmc_sq_c3d.txt $O/pmc_lds_c3d.txt | grep -v "^--" | head -60
fi
if [ -f flare-cpp_amd/lib/libflare_snappy_gpu_stamps.so ] && [ -z "$SKIP_STAMPS" ]; then
  timeout -k 10 120 python tools/stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
  cat $O/stamps.txt
fi
echo done
