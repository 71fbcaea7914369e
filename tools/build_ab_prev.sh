#!/bin/bash
# Builds the GPU codec library of a git revision (default HEAD) into
# build/ab/lib_prev.so for tools/gpurun/ab.sh's A/B pairs.
set -e
REV=${1:-HEAD}
D=$(mktemp -d)
git archive "$REV" flare-cpp_amd/csrc include | tar -x -C "$D"
mkdir -p build/ab
objs=""
for f in "$D"/flare-cpp_amd/csrc/*.hip; do
  o="$D/$(basename "$f" .hip).o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/lib_prev.so $objs
rm -rf "$D"
echo "build/ab/lib_prev.so <- $REV"
