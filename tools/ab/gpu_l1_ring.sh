#!/bin/bash
# Layer-1 (64 -> 64, 56x56) 3x3 conv: default engines vs the tap-ring engine (config 13) for
# the codes-only and residual epilogue forms.  Usage: bash tools/ab/gpu_l1_ring.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for F in "--no-out" "--residual"; do
  for C in 0 13; do
    timeout -k 10 120 python -u tools/conv_probe.py --layer 1 --config $C --codes 1 $F --iters 30 2>/dev/null | grep layer | sed "s/^/$F /" || exit 1
  done
done
