#!/bin/bash
# Staged-input wave encoder (small batches): parity, then the C1 echo with the
# stage on and off, then the kernel trace of the echo with it on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4stage
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread \
  -k "small_batch_wave_encoder or wave_encoder_against or golden" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for s in 1 0 1; do
  FSG_ENCODE_WAVE_STAGE=$s timeout -k 10 120 build/echo_bench --codec gpu --calls ${CALLS:-300} > $O/echo_s$s.json 2> $O/echo_s$s.err || { tail -5 $O/echo_s$s.err; exit 1; }
  echo "stage=$s"; head -c 600 $O/echo_s$s.json; echo
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o tr -- \
  build/echo_bench --codec gpu --calls ${CALLS:-300} > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
for f in $(find $O/tr -name "*kernel_stats.csv"); do echo "== $f"; head -12 $f; done
