#!/bin/bash
# A/B (candidate vs build/ab/lib_prev.so): GPU suite on the candidate, bench
# pairs on cm/c3/c2 and the 1 KiB / 4 KiB body sweep.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WLS="cm-decompress c3-decompress c2-decompress" bash tools/gpurun/ab.sh || exit 1
for lib in flare-cpp_amd/lib/libflare_snappy_gpu.so build/ab/lib_prev.so flare-cpp_amd/lib/libflare_snappy_gpu.so build/ab/lib_prev.so; do
  echo "== $lib"
  FSG_LIB=$lib timeout -k 10 200 python tools/size_sweep.py --sizes 1024,4096 > gpurun_out/ab/sweep.jsonl 2> gpurun_out/ab/sweep.err || { tail -5 gpurun_out/ab/sweep.err; exit 1; }
  cat gpurun_out/ab/sweep.jsonl
done
