#!/usr/bin/env bash
# A/B build of the kernel library with ONE source recompiled under extra
# flags (the other objects are the production ones from `make kernels`):
#
#   bash scripts/build_variant_lib.sh NAME SRC "FLAGS..."
#   -> mxk8s/_lib/libmxkernels_NAME.so   (select with MXK_KERNELS_LIB=...)
set -eu
cd "$(dirname "$0")/.."
name=$1 src=$2 flags=$3
make -s kernels
mkdir -p build/variant_$name
objs=()
for o in build/kernels/*.o; do
  b=$(basename "$o" .o)
  if [ "$b.hip" = "$(basename "$src")" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wshadow \
      -Wno-unused-function -Inative/kernels $flags -c "$src" -o build/variant_$name/$b.o
    objs+=(build/variant_$name/$b.o)
  else
    objs+=("$o")
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o mxk8s/_lib/libmxkernels_$name.so "${objs[@]}"
echo mxk8s/_lib/libmxkernels_$name.so
