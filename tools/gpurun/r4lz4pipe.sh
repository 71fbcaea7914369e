#!/bin/bash
# LZ4 two-stream form: GPU tests, then the C3 LZ4 bench (serial two-pass and
# the stream of two alternating batches).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4lz4pipe
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python tools/lz4_bench.py --steps 6 --two-pass-only --no-cpu > $O/lz4.json 2> $O/lz4.err || { tail -20 $O/lz4.err; exit 1; }
python -c "import json;d=json.load(open('$O/lz4.json'));print(json.dumps(d['decode_two_pass']));print(json.dumps(d['decode_two_pass_pipelined']))"
