#!/bin/bash
# Build timing-only ablation variants of libtq_hip.so (never loaded by the product: select
# one with TQ_LIB_PATH).  Usage: bash tools/ab/ablate.sh 1 2  -> lib/libtq_hip_abl1.so, ...
set -e
cd "$(dirname "$0")/../term-quantization_amd"
for V in "$@"; do
  mkdir -p build/abl$V
  for f in csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-gpu-rdc -DTQ_ABLATE=$V \
      -c $f -o build/abl$V/$(basename $f .hip).o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libtq_hip_abl$V.so build/abl$V/*.o
done
