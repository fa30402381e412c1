#!/bin/bash
# Timing-only ablations of the row-strip engine on layer 1 (conv1-style: codes out, no fp32):
# direct engine (TQ_STRIP=0), full strip, no epilogue (11), no MFMA (12), no team sync (13),
# no patch refill DMA (14), no main loop (15).  Usage: bash tools/gpu_ablate_strip.sh
set -u
L=${L:-1}
echo -n "direct: "; TQ_STRIP=0 timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --no-out --iters 20 2>/dev/null | tail -1 || exit 1
for V in ${VARS:-"" 11 12 13 14 15}; do
  lib=term-quantization_amd/lib/libtq_hip${V:+_abl$V}.so
  echo -n "strip abl '${V:-full}': "
  TQ_LIB_PATH=$(pwd)/$lib timeout -k 10 120 python tools/conv_probe.py --layer $L --codes 1 --no-out --iters 20 2>/dev/null | tail -1 || exit 1
done
