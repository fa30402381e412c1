#!/bin/bash
# MobileNet-V2 expand-conv shapes (1x1, small Cin -> large Cout, codes-only epilogue) on the
# direct engine (config 0 heuristic) and the expand engine (config 14).
# Usage: bash tools/gpu_expand_probe.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
for S in 16,96,1,1,112 24,144,1,1,56 32,192,1,1,28 64,384,1,1,14 96,576,1,1,14 160,960,1,1,7; do
  for C in 0 14; do
    timeout -k 10 120 python -u tools/conv_probe.py --shape $S --config $C --codes 1 --no-out --iters 20 2>/dev/null | grep layer | sed "s/^/$S /" || exit 1
  done
done
