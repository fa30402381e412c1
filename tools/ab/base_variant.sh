#!/bin/bash
# Build lib/libtq_hip_<name>.so from the csrc/ of a git revision (default HEAD), for A/B
# timing of working-tree kernel changes against it (select with TQ_LIB_PATH; never loaded by
# the product).  Usage: bash tools/ab/base_variant.sh [rev] [name]
set -e
REV=${1:-HEAD}; NAME=${2:-base}
cd "$(dirname "$0")/../term-quantization_amd"
T=$(mktemp -d)
mkdir -p $T/p/csrc $T/include build/var_$NAME  # csrc/ includes ../../include/tq.h
for f in $(git ls-tree --name-only $REV csrc/); do git show $REV:term-quantization_amd/$f > $T/p/$f; done
git show $REV:include/tq.h > $T/include/tq.h
for f in $T/p/csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-gpu-rdc \
    -c $f -o build/var_$NAME/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libtq_hip_$NAME.so build/var_$NAME/*.o
rm -rf $T
