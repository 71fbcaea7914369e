#!/bin/bash
# Pipelined (two-stream) C3 decode per library: libs in $LIBS (build/ab/lib_<name>.so).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe
mkdir -p $O
for lib in ${LIBS:-cur p6}; do
  for p in 1 0; do
    FSG_LIB=build/ab/lib_$lib.so timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-encode \
      --pipeline $p --verify-sample 8 > $O/${lib}_p$p.json 2> $O/${lib}_p$p.err || { tail -5 $O/${lib}_p$p.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${lib}_p$p.json'));print('$lib pipe=$p', d['ms_per_step'], d.get('pipeline'), d['correct'])"
  done
done
