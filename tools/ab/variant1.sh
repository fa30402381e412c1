#!/bin/bash
# Build a timing variant of libtq_hip.so that recompiles ONE kernel source with extra flags and
# links it with the product objects of the others (never loaded by the product: select it with
# TQ_LIB_PATH).  Usage: bash tools/ab/variant1.sh NAME SOURCE "-DFOO=1 ..."
#   -> term-quantization_amd/lib/libtq_hip_NAME.so
set -e
cd "$(dirname "$0")/../term-quantization_amd"
NAME=$1; SRC=$2; shift 2
mkdir -p build/var_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-gpu-rdc -munsafe-fp-atomics $* \
  -c csrc/$SRC.hip -o build/var_$NAME/$SRC.o 2>/dev/null
OBJS=""
for o in build/*.o; do
  b=$(basename $o)
  if [ "$b" = "$SRC.o" ]; then OBJS="$OBJS build/var_$NAME/$SRC.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libtq_hip_$NAME.so $OBJS
