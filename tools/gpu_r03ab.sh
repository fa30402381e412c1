#!/bin/bash
# r03ab: MobileNet-V2 1x1 shapes on the direct engine, 64-row (config 10) vs 128-row (9) tiles
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r03ab}; O=gpurun_out/$TAG; mkdir -p $O
for A in "16,96,1,1,112" "24,144,1,1,56" "32,192,1,1,28" "64,384,1,1,14" "96,576,1,1,14" "160,960,1,1,7" "144,24,1,1,56" "192,32,1,1,28" "32,16,1,1,112"; do
  for C in 10 9; do
    echo -n "$A cfg $C: "; timeout -k 10 120 python tools/conv_probe.py --shape $A --codes 1 --no-out --config $C --iters 20 2>>$O/err.log | tail -1 || echo fail
  done
done | tee $O/tiles.txt
