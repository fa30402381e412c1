#!/bin/bash
# MobileNet-V2 / EfficientNet-b0 expand-conv shapes (1x1, small Cin -> large Cout, codes-only
# epilogue): config 0 (the heuristic, which picks the expand engine for these shapes) and 10
# (the direct engine), optionally against a variant build.  Usage: bash tools/ab/gpu_expand_probe.sh [variant]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; V=${1:-}
for S in 16,96,1,1,112 24,144,1,1,56 32,192,1,1,28 40,240,1,1,28 64,384,1,1,14 80,480,1,1,14 96,576,1,1,14 112,672,1,1,14 160,960,1,1,7; do
  for C in 0 10; do
    timeout -k 10 120 python -u tools/conv_probe.py --shape $S --config $C --codes 1 --no-out --iters 20 2>/dev/null | grep layer | sed "s/^/$S /" || exit 1
  done
  if [ -n "$V" ]; then
    TQ_LIB_PATH=$R/term-quantization_amd/lib/libtq_hip_$V.so timeout -k 10 120 python -u tools/conv_probe.py --shape $S --config 0 --codes 1 --no-out --iters 20 2>/dev/null | grep layer | sed "s/^/$S $V /" || exit 1
  fi
done
