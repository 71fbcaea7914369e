#!/bin/bash
# Round 4: wave encoder parity, then compress A/B over configurations
# CFGS="name:VAR=v,VAR2=v ..." (default: lane encoder vs wave encoder for
# messages >= 16 KiB), optional stamps / kernel stats, then the GPU suite.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "wave_encoder" > $O/pytest_wave.log 2>&1 || { tail -40 $O/pytest_wave.log; exit 1; }
tail -3 $O/pytest_wave.log
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --verify-sample 16"
for w in ${WLS:-c3-compress c5-compress}; do
  for cfg in ${CFGS:-lane:FSG_ENCODE_WAVE_MIN=0 wave:FSG_ENCODE_WAVE_MIN=16384}; do
    name=${cfg%%:*}; envs=$(echo ${cfg#*:} | tr ',' ' ')
    env $envs timeout -k 10 300 $B --workload $w > $O/bench_${w}_$name.json 2> $O/bench_${w}_$name.err \
      || { tail -20 $O/bench_${w}_$name.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${w}_$name.json'));print('$w $name', d['ms_per_step'], d['value'], d['correct'])"
  done
done
if [ -n "$WSTAMPS" ]; then
  timeout -k 10 200 python tools/wstamps.py 16384 > $O/wstamps.txt 2>&1 || { tail -20 $O/wstamps.txt; exit 1; }
  cat $O/wstamps.txt
fi
if [ -n "$KST" ]; then
  for w in c5-compress c3-compress; do
    rm -rf $O/kst_$w
    FSG_ENCODE_WAVE_MIN=${KST_WAVE_MIN:-16384} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kst_$w -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --verify-sample 0 --workload $w > $O/kst_$w.log 2>&1 || { tail -5 $O/kst_$w.log; exit 1; }
    python - "$(find $O/kst_$w -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "fsg::" in r["Name"]:
        print(r["Name"].split("(")[0][:60], r["Calls"], "%.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
  done
fi
[ -n "$SKIP_SUITE" ] || bash tools/gpurun/r4t.sh
