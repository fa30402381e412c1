#!/bin/bash
# Timing-only ablations of the input-patch engine (lib/libtq_hip_ablN.so, tools/ablate.sh):
# full kernel vs no fragment reads (1), no MFMA (2), no LDS-DMA (3), no barrier (4),
# setup + epilogue only (6), no epilogue stores (7), on layers 11 and 16 (conv1-style: codes
# out, no fp32).  Usage: bash tools/gpu_ablate_patch.sh <tag>
set -u
O=gpurun_out/${1:-abl}
mkdir -p $O
for L in 11 16; do
  for V in "" 1 2 3 4 6 7; do
    lib=term-quantization_amd/lib/libtq_hip${V:+_abl$V}.so
    echo -n "layer $L abl '${V:-full}': "
    TQ_LIB_PATH=$(pwd)/$lib timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --no-out --iters 20 2>/dev/null | tail -1 || exit 1
  done
done
