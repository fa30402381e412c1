#!/bin/bash
# Build libtq_hip with extra compile flags into term-quantization_amd/lib/libtq_hip_<name>.so
# (a separate object directory; A/B runs load it through TQ_LIB_PATH).
# Usage: bash tools/ab/build_variant.sh <name> "<extra hipcc flags>"
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
NAME=$1; EXTRA=$2
P=$R/term-quantization_amd
B=/tmp/tq_build_$NAME
mkdir -p $B
cd $P
SRCS=$(sed -n 's/^SRCS = //p' Makefile)
for s in $SRCS; do
  o=$B/$(basename ${s%.hip}).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
      -fno-gpu-rdc -munsafe-fp-atomics $EXTRA -c $s -o $o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libtq_hip_$NAME.so $B/*.o
ls -la lib/libtq_hip_$NAME.so
