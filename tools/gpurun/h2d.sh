#!/bin/bash
# The default bench line's end-to-end leg, twice, for the H2D diagnosis.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/h2d; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-encode --verify-sample 0 \
    > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b$i.json'))['end_to_end'];print({k:d[k] for k in ('h2d_gb_s','h2d_gb_s_host_clock','h2d_gb_s_diag','d2h_gb_s')})"
done
