#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4t2; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
