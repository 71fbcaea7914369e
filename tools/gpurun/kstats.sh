#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) for each build/ab/lib_<name>.so
# entry of $LIBS (name@VAR=value sets an environment variable), on $WLS.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kst
for w in ${WLS:-c3-decompress}; do
  for e in $LIBS; do
    n=${e%%@*}; env_kv=""; [ "$e" != "$n" ] && env_kv=${e#*@}
    tag=$(echo "$e" | tr '@=' '__')_$w
    rm -rf gpurun_out/kst/$tag
    env $env_kv FSG_LIB=build/ab/lib_$n.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kst/$tag -o run -- \
      python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-encode --verify-sample 0 --workload $w \
      > gpurun_out/kst/$tag.log 2>&1 || { tail -5 gpurun_out/kst/$tag.log; exit 1; }
    f=$(find gpurun_out/kst/$tag -name "*kernel_stats.csv" | head -1)
    python - "$f" "$tag" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Name"].startswith("fsg::")]
print(sys.argv[2], " ".join("%s=%.3f" % (r["Name"].split("(")[0].replace("fsg::", ""), float(r["AverageNs"]) / 1e6) for r in rows))
PY
  done
done
