#!/bin/bash
# GPU parity suite on the in-tree build, then an N-way A/B (tools/gpurun/abn.sh).
mkdir -p gpurun_out/abn
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/abn/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/abn/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/abn/pytest_gpu.log
bash tools/gpurun/abn.sh
