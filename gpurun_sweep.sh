#!/bin/bash
# smoke() + exec_kernel large-block-count sweep on C3 and CM (one box).
mkdir -p gpurun_out/sweep
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/sweep/smoke.log 2>&1 || { tail -20 gpurun_out/sweep/smoke.log; exit 1; }
tail -1 gpurun_out/sweep/smoke.log
B="python bench.py --no-cpu-baseline --no-e2e --steps 10 --warmup 2 --verify-sample 16"
for w in c3-decompress cm-decompress; do
  for nb in 128 512 256 1024 128 512; do
    FSG_EXEC_BIG_BLOCKS=$nb timeout -k 10 240 $B --workload $w > gpurun_out/sweep/$w_$nb.json 2> gpurun_out/sweep/err.log || { tail -5 gpurun_out/sweep/err.log; exit 1; }
    echo "$w $nb $(python -c "import json;d=json.load(open('gpurun_out/sweep/$w_$nb.json'));print(d['ms_per_step'], d['correct']['status_errors'])")"
  done
done
