#!/bin/bash
# N-way A/B on one box: each build/ab/lib_<name>.so in $LIBS, interleaved
# twice over, on the workloads in $WLS (default C3 decode).  An entry
# name@VAR=value runs lib_<name>.so with that environment variable set.
mkdir -p gpurun_out/abn
B="python bench.py --no-cpu-baseline --no-e2e --no-encode --pipeline 0 --steps 10 --warmup 2 --verify-sample 16"
for w in ${WLS:-c3-decompress}; do
  for pass in 1 2; do
    for e in $LIBS; do
      n=${e%%@*}; env_kv=""; [ "$e" != "$n" ] && env_kv=${e#*@}
      tag=$(echo "$e" | tr '@=' '__')
      env $env_kv FSG_LIB=build/ab/lib_$n.so timeout -k 10 240 $B --workload $w > gpurun_out/abn/${tag}_${w}_$pass.json 2> gpurun_out/abn/${tag}_${w}_$pass.err || { tail -5 gpurun_out/abn/${tag}_${w}_$pass.err; exit 1; }
      echo "$e $w $(python -c "import json;d=json.load(open('gpurun_out/abn/${tag}_${w}_$pass.json'));print(d['ms_per_step'], d['correct']['oracle_sample_ok'], d['correct']['status_errors'])")"
    done
  done
done
