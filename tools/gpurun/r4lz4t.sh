#!/bin/bash
# LZ4 two-pass decode: GPU parity, then the kernel split (r4lz4p.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4lz4p
timeout -k 10 300 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4lz4p/pytest.log 2>&1 || { tail -40 gpurun_out/r4lz4p/pytest.log; exit 1; }
tail -2 gpurun_out/r4lz4p/pytest.log
bash tools/gpurun/r4lz4p.sh "$@"
