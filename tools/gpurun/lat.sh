#!/bin/bash
# Item 5: account for one single-message device batch.  The echo
# bench with every body on the GPU, under the kernel + HIP API trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${OUT:-gpurun_out/lat}
rm -rf $O; mkdir -p $O
timeout -k 10 120 build/echo_bench --codec gpu --calls ${CALLS:-200} > $O/echo_gpu.json 2> $O/echo_gpu.err || { tail -5 $O/echo_gpu.err; exit 1; }
cat $O/echo_gpu.json | head -c 1500; echo
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $O/tr -o tr -- \
  build/echo_bench --codec gpu --calls ${CALLS:-200} > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
ls $O/tr/*/ | head
for f in $(find $O/tr -name "*kernel_stats.csv" -o -name "*hip_api_stats.csv"); do echo "== $f"; head -25 $f; done
