#!/bin/bash
# Builds build/ab/lib_<name>.so for each "name:FLAGS" argument (the current
# tree's GPU sources with extra -D flags), for tools/gpurun/abn.sh.
set -e
mkdir -p build/ab
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  D=build/ab/obj_$name; mkdir -p $D
  objs=""
  for f in flare-cpp_amd/csrc/*.hip; do
    o=$D/$(basename $f .hip).o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c $f -o $o &
    objs="$objs $o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/lib_$name.so $objs
  echo "build/ab/lib_$name.so [$flags]"
done
