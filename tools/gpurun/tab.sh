#!/bin/bash
# GPU parity suite (unless SKIP_TESTS), then the N-way A/B of abn.sh.
# usage: LIBS="cur base" WLS="c3-decompress" bash tools/gpurun/tab.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tab
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/tab/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/tab/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/tab/pytest_gpu.log
fi
bash tools/gpurun/abn.sh
