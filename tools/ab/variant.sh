#!/bin/bash
# Build a timing variant of libtq_hip.so with extra compile flags (never loaded by the
# product: select it with TQ_LIB_PATH).  Usage: bash tools/ab/variant.sh NAME "-DFOO=1 ..."
#   -> term-quantization_amd/lib/libtq_hip_NAME.so
set -e
cd "$(dirname "$0")/../term-quantization_amd"
NAME=$1; shift
mkdir -p build/var_$NAME
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-gpu-rdc $* \
    -c $f -o build/var_$NAME/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libtq_hip_$NAME.so build/var_$NAME/*.o
