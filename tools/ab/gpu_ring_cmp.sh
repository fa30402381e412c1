#!/bin/bash
# Ring shapes side by side: per-layer timings of the default engines, shape 1 and shape 2 for
# both epilogue forms.  Usage: bash tools/ab/gpu_ring_cmp.sh <tag> "<layers>"
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-cmp}; LAYERS=${2:-"6 8 11 13 16 18"}
for L in $LAYERS; do
  for F in "--residual" "--no-out"; do
    timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 0 --codes 1 $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F base /" || exit 1
    for V in 1 2; do
      TQ_RING_V=$V timeout -k 10 120 python -u tools/conv_probe.py --layer $L --config 13 --codes 1 $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F v$V /" || exit 1
    done
  done
done
