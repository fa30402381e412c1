#!/bin/bash
# Ring-engine timing ablations (libtq_hip_<variant>.so) for both epilogue forms.
# Usage: bash tools/ab/gpu_ring_ab2.sh "<layers>" "<variants>"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; LAYERS=$1; VARS=$2
for L in $LAYERS; do
  for F in "--no-out" "--residual"; do
    for v in default $VARS; do
      lib=""; [ "$v" != default ] && lib=$R/term-quantization_amd/lib/libtq_hip_$v.so
      TQ_LIB_PATH=$lib timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 13 --codes 1 --nonneg $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F $v /" || exit 1
    done
  done
done
