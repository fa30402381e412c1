#!/bin/bash
# Timing-only ablations of the direct engine (lib/libtq_hip_ablN.so, tools/ablate.sh 2 3 6 7):
# full kernel vs no MFMA (2), no A-DMA / B loads (3), setup + epilogue only (6), no epilogue
# stores (7), on ResNet-18 layers 6 (conv1-style: codes out) and 8 / 2 (conv2-style: fp32 out
# + codes + fp32 residual in).  Usage: bash tools/gpu_ablate_direct.sh <tag>
set -u
O=gpurun_out/${1:-ablD}
mkdir -p $O
for spec in "6:--codes 1 --no-out" "8:--codes 1 --residual" "2:--codes 1 --residual"; do
  L=${spec%%:*}; A=${spec#*:}
  for V in "" 2 3 6 7; do
    lib=term-quantization_amd/lib/libtq_hip${V:+_abl$V}.so
    echo -n "layer $L [$A] abl '${V:-full}': "
    TQ_STRIP=0 TQ_LIB_PATH=$(pwd)/$lib timeout -k 10 120 python tools/conv_probe.py --layer $L $A --iters 20 2>/dev/null | tail -1 || exit 1
  done
done
